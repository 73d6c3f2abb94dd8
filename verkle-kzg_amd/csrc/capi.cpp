// extern "C" entry points of libvkzg.so (declared in include/vc_msm.h).
#include <algorithm>
#include <atomic>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "ctx.hpp"

namespace vk {

hipError_t& last_hip_error() {
    static thread_local hipError_t e = hipSuccess;
    return e;
}

// pooled blocks: best fit within 2x (+1 MiB) of the request; at most VK_POOL_MAX cached bytes
constexpr size_t VK_POOL_MAX = 16ull << 30;

int pool_take(vc_ctx* ctx, size_t bytes, void** p, size_t* cap) {
    auto it = ctx->pool_free.lower_bound(bytes);
    if (it != ctx->pool_free.end() && it->first <= 2 * bytes + (1u << 20)) {
        *p = it->second;
        *cap = it->first;
        ctx->pool_bytes -= it->first;
        ctx->pool_free.erase(it);
        return VC_OK;
    }
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory && !ctx->pool_free.empty()) {  // give the cached blocks back, retry
        (void)hipGetLastError();
        for (auto& kv : ctx->pool_free) (void)hipFree(kv.second);
        ctx->pool_free.clear();
        ctx->pool_bytes = 0;
        e = hipMalloc(p, bytes);
    }
    if (e != hipSuccess) {
        last_hip_error() = e;
        *p = nullptr;
        *cap = 0;
        return VC_E_OOM;
    }
    *cap = bytes;
    return VC_OK;
}

void pool_put(vc_ctx* ctx, void* p, size_t cap) {
    if (ctx->pool_bytes + cap > VK_POOL_MAX) {
        (void)hipFree(p);
        return;
    }
    ctx->pool_free.emplace(cap, p);
    ctx->pool_bytes += cap;
}

// live contexts by uid: a verkle tree's device mirror outlives the calls that use it and goes back
// to its context's pool when released -- if that context still exists and is not busy
namespace {
std::mutex g_live_mu;
std::unordered_map<uint64_t, vc_ctx*>& live_ctx() {
    static std::unordered_map<uint64_t, vc_ctx*> m;
    return m;
}
}  // namespace
void ctx_register(vc_ctx* ctx, bool live) {
    std::lock_guard<std::mutex> lk(g_live_mu);
    if (live) live_ctx()[ctx->uid] = ctx;
    else live_ctx().erase(ctx->uid);
}
void pool_return_uid(uint64_t uid, int dev, void* p, size_t cap) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_live_mu);
        auto it = live_ctx().find(uid);
        // (try_lock: another thread may hold the context's lock, then the block is freed; the
        // calling thread may hold it too -- the lock is recursive, so that try_lock succeeds)
        if (it != live_ctx().end() && it->second->mu.try_lock()) {
            pool_put(it->second, p, cap);
            it->second->mu.unlock();
            return;
        }
    }
    DeviceScope on(dev);  // hipFree on the block's device; the caller's current device is restored
    (void)hipFree(p);
}

int DevBuf::ensure(size_t bytes) {
    if (bytes <= cap && p) return VC_OK;
    release();
    if (bytes == 0) bytes = 16;
    if (pool) return pool_take(pool, bytes, &p, &cap);
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        last_hip_error() = e;
        p = nullptr;
        cap = 0;
        return VC_E_OOM;
    }
    cap = bytes;
    return VC_OK;
}

int PinBuf::ensure(size_t bytes) {
    if (bytes <= cap && p) return VC_OK;
    // grow by half at least (and to 64 KiB): a page-locked re-allocation costs ~0.1-0.3 ms, and
    // callers whose sizes creep up call by call (the verkle levels of successive updates) would
    // otherwise pay it again and again
    if (p) bytes = std::max(bytes, cap + cap / 2);
    bytes = std::max<size_t>(bytes, 64 << 10);
    release();
    hipError_t e = hipHostMalloc(&p, bytes, flags ? flags : hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dp, p, 0);
    if (e != hipSuccess) {
        last_hip_error() = e;
        if (p) (void)hipHostFree(p);
        p = dp = nullptr;
        cap = 0;
        return VC_E_OOM;
    }
    cap = bytes;
    return VC_OK;
}

void PinBuf::release() {
    if (p) (void)hipHostFree(p);
    p = dp = nullptr;
    cap = 0;
}

void DevBuf::release() {
    if (p && pool) pool_put(pool, p, cap);
    else if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
}

}  // namespace vk

hipEvent_t vc_ctx::get_event() {
    if (!event_pool.empty()) {
        hipEvent_t e = event_pool.back();
        event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

void vc_ctx::timer_begin(const char*, hipEvent_t* a, hipStream_t s) {
    *a = get_event();
    (void)hipEventRecord(*a, s ? s : stream);
}

void vc_ctx::timer_end(const char* name, hipEvent_t a, hipStream_t s) {
    hipEvent_t b = get_event();
    (void)hipEventRecord(b, s ? s : stream);
    pending.push_back({a, b, name});
}

uint64_t* vc_ctx::clk_slot() {
    constexpr uint32_t SLOTS = 256;
    const bool fresh = clk.p == nullptr;
    if (!timing || clk.ensure(SLOTS * 4 * sizeof(uint64_t)) != VC_OK) return nullptr;
    if (fresh && (hipMemsetAsync(clk.p, 0, clk.cap, stream) != hipSuccess || hipStreamSynchronize(stream) != hipSuccess))
        return nullptr;
    if (clk_pending.size() >= SLOTS) return nullptr;  // uncollected slots would be overwritten
    const uint32_t s = clk_next++ % SLOTS;
    clk_pending.push_back(s);
    return clk.as<uint64_t>() + 4 * (size_t)s;
}

void vc_ctx::collect_timers() {
    if (!clk_pending.empty()) {
        // the stamping kernels ran on the context's (non-blocking) streams: wait for both before the
        // read-back, and clear the slots after it, so a reused slot never shows an older launch
        (void)hipStreamSynchronize(stream);
        (void)hipStreamSynchronize(side_stream);
        std::vector<uint64_t> h(clk.cap / sizeof(uint64_t));
        const bool ok = hipMemcpyAsync(h.data(), clk.p, clk.cap, hipMemcpyDeviceToHost, stream) == hipSuccess &&
                        hipMemsetAsync(clk.p, 0, clk.cap, stream) == hipSuccess &&
                        hipStreamSynchronize(stream) == hipSuccess;
        if (ok)
            for (uint32_t s : clk_pending) {
                const uint64_t* v = &h[4 * (size_t)s];
                if (v[2] > v[0] && v[3] > v[1]) {
                    clk_cycles += (double)(v[2] - v[0]);
                    clk_ticks += (double)(v[3] - v[1]);
                    clk_n++;
                }
            }
        clk_pending.clear();
    }
    for (auto& p : pending) {
        float ms = 0.f;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            auto& slot = ktime[p.name];
            slot.first += ms;
            slot.second += 1;
        }
        event_pool.push_back(p.a);
        event_pool.push_back(p.b);
    }
    pending.clear();
}

namespace {

struct Guard {
    vc_ctx* c;
    std::lock_guard<std::recursive_mutex> lk;
    explicit Guard(vc_ctx* ctx) : c(ctx), lk(ctx->mu) { (void)hipSetDevice(ctx->device); }
    ~Guard() {
        if (c->timing) c->collect_timers();
    }
};

bool valid_curve(int c) { return c == VC_CURVE_BN254 || c == VC_CURVE_BLS12_381 || c == VC_CURVE_BANDERSNATCH; }

}  // namespace

extern "C" {

const char* vc_strerror(int s) {
    switch (s) {
        case VC_OK: return "ok";
        case VC_E_INVALID: return "invalid argument";
        case VC_E_HIP: return hipGetErrorString(vk::last_hip_error());
        case VC_E_OOM: return "device out of memory";
        case VC_E_TABLE: return "unknown or incompatible base table";
        case VC_E_RANGE: return "range beyond the base table";
        case VC_E_NOT_ON_CURVE: return "base point not on the curve (or not canonical)";
        case VC_E_NO_DEVICE: return "no usable HIP device";
        case VC_E_DOMAIN: return "evaluation point outside the supported domain";
        case VC_E_COMM: return "collective failed (RCCL or the all-gather callback)";
        case VC_E_PEER: return "another rank of the group failed this step";
    }
    return "unknown status";
}

int vc_version(void) { return 1; }

int vc_device_mad_rate(vc_ctx* ctx, double* tera_per_s) {
    if (!ctx || !tera_per_s) return VC_E_INVALID;
    Guard g(ctx);
    return vk::device_mad_rate(ctx, tera_per_s);
}

int vc_ctx_create(int curve, int device, vc_ctx** out) {
    if (!out || !valid_curve(curve)) return VC_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return VC_E_NO_DEVICE;
    if (device < 0 || device >= ndev) return VC_E_INVALID;
    VK_CHECK_HIP(hipSetDevice(device));
    vc_ctx* c = new vc_ctx();
    static std::atomic<uint64_t> next_uid{1};
    c->uid = next_uid.fetch_add(1);
    c->curve = curve;
    c->device = device;
    c->pin_small.flags = hipHostMallocCoherent;
    c->pin_norm_vk.flags = hipHostMallocCoherent;  // written by kernels, polled by the host
    c->pin[0].flags = c->pin[1].flags = hipHostMallocCoherent;  // the MSM tails' points and flags
    hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        vk::last_hip_error() = e;
        delete c;
        return VC_E_HIP;
    }
    e = hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        vk::last_hip_error() = e;
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return VC_E_HIP;
    }
    c->stream = c->own_stream;
    vk::ctx_register(c, true);
    *out = c;
    return VC_OK;
}

void vc_ctx_destroy(vc_ctx* ctx) {
    if (!ctx) return;
    vk::ctx_register(ctx, false);  // before its lock: no mirror block comes back to it after this
    {
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        (void)hipSetDevice(ctx->device);
        if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
        for (auto* t : ctx->tables) delete t;
        ctx->tables.clear();
        for (auto& b : ctx->ws) b.release();
        for (auto& b : ctx->ws2) b.release();
        for (auto& b : ctx->pin) b.release();
        ctx->pin_io.release();
        ctx->pin_small.release();
        ctx->pin_norm.release();
        ctx->pin_y.release();
        ctx->pin_mp.release();
        ctx->pin_ipa.release();
        ctx->pin_verkle.release();
        ctx->pin_verkle2.release();
        for (auto& b : ctx->pin_verkle_lv) b.release();
        ctx->pin_norm_vk.release();
        ctx->pin_sparse_ck.release();
        ctx->pin_sparse_ch.release();
        for (auto& kv : ctx->pool_free) (void)hipFree(kv.second);
        ctx->pool_free.clear();
        for (auto& p : ctx->pending) {
            (void)hipEventDestroy(p.a);
            (void)hipEventDestroy(p.b);
        }
        for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
        if (ctx->side_stream) {
            (void)hipStreamSynchronize(ctx->side_stream);
            (void)hipStreamDestroy(ctx->side_stream);
        }
        if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    }
    delete ctx;
}

int vc_ctx_curve(const vc_ctx* ctx) { return ctx ? ctx->curve : VC_E_INVALID; }

int vc_ctx_set_stream(vc_ctx* ctx, void* s) {
    if (!ctx) return VC_E_INVALID;
    Guard g(ctx);
    hipStream_t ns = s ? reinterpret_cast<hipStream_t>(s) : ctx->own_stream;
    // pooled scratch freed by work still queued on the old stream must not be reused on the new one
    if (ns != ctx->stream && ctx->stream) VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    ctx->stream = ns;
    return VC_OK;
}

int vc_ctx_set_option(vc_ctx* ctx, int option, int64_t value) {
    if (!ctx) return VC_E_INVALID;
    Guard g(ctx);
    switch (option) {
        case VC_OPT_MSM_SHARED_WINDOWS:
            ctx->opt_shared_windows = value != 0;
            return VC_OK;
        case VC_OPT_MSM_CHUNK_POINTS:
            if (value < 1 || value > (int64_t(1) << 27)) return VC_E_INVALID;
            ctx->opt_msm_chunk = (size_t)value;
            return VC_OK;
        case VC_OPT_MSM_HOST_CHUNKS:
            if (value < 1 || value > 4) return VC_E_INVALID;
            ctx->opt_host_chunks = (int)value;
            return VC_OK;
    }
    return VC_E_INVALID;
}

int vc_ctx_get_option(vc_ctx* ctx, int option, int64_t* value) {
    if (!ctx || !value) return VC_E_INVALID;
    Guard g(ctx);
    switch (option) {
        case VC_OPT_MSM_SHARED_WINDOWS: *value = ctx->opt_shared_windows; return VC_OK;
        case VC_OPT_MSM_CHUNK_POINTS: *value = (int64_t)ctx->opt_msm_chunk; return VC_OK;
        case VC_OPT_MSM_HOST_CHUNKS: *value = ctx->opt_host_chunks; return VC_OK;
    }
    return VC_E_INVALID;
}

int vc_ctx_enable_timing(vc_ctx* ctx, int on) {
    if (!ctx) return VC_E_INVALID;
    Guard g(ctx);
    ctx->timing = on != 0;
    return VC_OK;
}

int vc_ctx_kernel_time(vc_ctx* ctx, const char* name, double* total_ms, long* launches) {
    if (!ctx || !name) return VC_E_INVALID;
    Guard g(ctx);
    auto it = ctx->ktime.find(name);
    if (total_ms) *total_ms = it == ctx->ktime.end() ? 0.0 : it->second.first;
    if (launches) *launches = it == ctx->ktime.end() ? 0 : it->second.second;
    return VC_OK;
}

int vc_ctx_accumulate_clock(vc_ctx* ctx, double* mhz, long* launches) {
    if (!ctx || !mhz) return VC_E_INVALID;
    Guard g(ctx);
    *mhz = ctx->clk_ticks > 0 ? ctx->clk_cycles / ctx->clk_ticks * 100.0 : 0.0;
    if (launches) *launches = ctx->clk_n;
    return VC_OK;
}

int vc_ctx_reset_timing(vc_ctx* ctx) {
    if (!ctx) return VC_E_INVALID;
    Guard g(ctx);
    ctx->ktime.clear();
    ctx->clk_cycles = ctx->clk_ticks = 0.0;
    ctx->clk_n = 0;
    return VC_OK;
}

int vc_bases_upload(vc_ctx* ctx, const uint64_t* xy, const uint8_t* inf, size_t n, int* id) {
    if (!ctx || !id || (n > 0 && !xy) || n >= 0x7fffffffu) return VC_E_INVALID;
    Guard g(ctx);
    return vk::bases_upload(ctx, xy, inf, n, id);
}

int vc_bases_count(vc_ctx* ctx, int id, size_t* n) {
    if (!ctx || !n) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    *n = t->n;
    return VC_OK;
}

int vc_bases_random(vc_ctx* ctx, uint64_t seed, size_t n, int* id) {
    if (!ctx || !id || n >= 0x7fffffffu) return VC_E_INVALID;
    Guard g(ctx);
    return vk::bases_random(ctx, seed, n, id);
}

int vc_bases_download(vc_ctx* ctx, int id, uint64_t* xy, uint8_t* inf) {
    if (!ctx || !xy) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    return vk::bases_download(ctx, t, xy, inf);
}

int vc_point_words(int curve) { return valid_curve(curve) ? vk::point_words(curve) : VC_E_INVALID; }

static int msm_device_acc(vc_ctx* ctx, int id, size_t offset, const void* d_sc, size_t n, int mont,
                          uint32_t* acc, int part = 0, int parts = 1) {
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    if (offset > t->n || n > t->n - offset) return VC_E_RANGE;
    if (n > 0 && !d_sc) return VC_E_INVALID;
    return vk::msm_run(ctx, t, offset, d_sc, n, mont, acc, part, parts);
}

int vc_msm_windows(int curve, size_t n, int* window_bits, int* windows, int* terms_per_point) {
    if (!valid_curve(curve) || !window_bits || !windows) return VC_E_INVALID;
    return vk::msm_windows(curve, n, window_bits, windows, terms_per_point);
}

int vc_msm_last_plan(const vc_ctx* ctx, int* window_bits, int* windows, int* terms_per_point, int* radix_mul,
                     int* shared_windows) {
    if (!ctx) return VC_E_INVALID;
    if (window_bits) *window_bits = ctx->plan.c;
    if (windows) *windows = ctx->plan.W;
    if (terms_per_point) *terms_per_point = ctx->plan.terms;
    if (radix_mul) *radix_mul = ctx->plan.m;
    if (shared_windows) *shared_windows = ctx->plan.shared;
    return VC_OK;
}

int vc_msm_device_window_part(vc_ctx* ctx, int id, size_t offset, const void* d_sc, size_t n, int mont, int part,
                              int parts, uint32_t* out_acc) {
    if (!ctx || !out_acc || parts < 1 || part < 0 || part >= parts) return VC_E_INVALID;
    Guard g(ctx);
    return msm_device_acc(ctx, id, offset, d_sc, n, mont, out_acc, part, parts);
}

int vc_msm_device_partial(vc_ctx* ctx, int id, size_t offset, const void* d_sc, size_t n, int mont,
                          uint32_t* out_acc) {
    if (!ctx || !out_acc) return VC_E_INVALID;
    Guard g(ctx);
    return msm_device_acc(ctx, id, offset, d_sc, n, mont, out_acc);
}

int vc_msm_device(vc_ctx* ctx, int id, size_t offset, const void* d_sc, size_t n, int mont,
                  uint64_t* out_xy, uint8_t* out_inf) {
    if (!ctx || !out_xy || !out_inf) return VC_E_INVALID;
    Guard g(ctx);
    std::vector<uint32_t> acc(vk::point_words(ctx->curve));
    VK_TRY(msm_device_acc(ctx, id, offset, d_sc, n, mont, acc.data()));
    static const bool timing = getenv("VKZG_HOST_TIMING") && atoi(getenv("VKZG_HOST_TIMING")) != 0;
    if (!timing) return vk::acc_to_affine(ctx->curve, acc.data(), out_xy, out_inf);
    const auto a0 = std::chrono::steady_clock::now();
    const int st = vk::acc_to_affine(ctx->curve, acc.data(), out_xy, out_inf);
    fprintf(stderr, "msm_affine_us=%.1f\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a0).count());
    return st;
}

int vc_msm_device_many(vc_ctx* ctx, int id, const void* const* d_scalars, const int* mont, size_t n, size_t count,
                       uint64_t* out_xy, uint8_t* out_inf) {
    if (!ctx || (count && (!d_scalars || !mont || !out_xy || !out_inf))) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    if (n > t->n) return VC_E_RANGE;
    for (size_t k = 0; k < count; k++)
        if (n > 0 && !d_scalars[k]) return VC_E_INVALID;
    if (count == 0) return VC_OK;
    const int words = vk::point_words(ctx->curve);
    std::vector<uint32_t> acc((size_t)words * count);
    VK_TRY(vk::msm_run_many(ctx, t, d_scalars, mont, n, count, acc.data()));
    const int NL = vk::aff_limbs64(ctx->curve);
    for (size_t k = 0; k < count; k++)
        VK_TRY(vk::acc_to_affine(ctx->curve, acc.data() + k * words, out_xy + k * 2 * NL, out_inf + k));
    return VC_OK;
}

// batched fixed-base commits of host scalars over bases [0, width) (vc_msm_batch; the caller holds
// the ctx lock)
static int batch_commit_host(vc_ctx* ctx, vk::Table* t, size_t width, const uint64_t* scalars, size_t batch, int mont,
                             uint64_t* out_xy, uint8_t* out_inf) {
    if (batch == 0) return VC_OK;
    const size_t nl = (size_t)vk::aff_limbs64(ctx->curve);
    VK_TRY(ctx->ws[vk::WS_SCALARS].ensure(batch * width * 32));
    VK_TRY(ctx->ws[vk::WS_MISC].ensure(batch * (2 * nl * 8 + 1)));
    uint8_t* dxy = ctx->ws[vk::WS_MISC].as<uint8_t>();
    uint8_t* dinf = dxy + batch * 2 * nl * 8;
    VK_CHECK_HIP(hipMemcpyAsync(ctx->ws[vk::WS_SCALARS].p, scalars, batch * width * 32,
                                hipMemcpyHostToDevice, ctx->stream));
    bool on_host = false;
    VK_TRY(vk::msm_batch_run(ctx, t, width, ctx->ws[vk::WS_SCALARS].p, batch, mont, dxy, dinf, out_xy, out_inf,
                             &on_host));
    if (on_host) return VC_OK;
    VK_CHECK_HIP(hipMemcpyAsync(out_xy, dxy, batch * 2 * nl * 8, hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipMemcpyAsync(out_inf, dinf, batch, hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}

int vc_msm(vc_ctx* ctx, int id, size_t offset, const uint64_t* scalars, size_t n, int mont,
           uint64_t* out_xy, uint8_t* out_inf) {
    if (!ctx || !out_xy || !out_inf || (n > 0 && !scalars)) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    if (offset > t->n || n > t->n - offset) return VC_E_RANGE;
    // a small MSM from the start of a table whose fixed-base windows the caller precomputed
    // (vc_fixed_base_precompute over a CRS at setup): the fixed-base latency path -- one (base,
    // window) point per thread, quad-add block sums -- instead of the Pippenger pipeline's fixed
    // ~0.25 ms (IPA::commit at width 256 through vc_msm: the reference's commit)
    if (n > 0 && n <= 1024 && offset == 0 && t->fb_c != 0)
        return batch_commit_host(ctx, t, n, scalars, 1, mont, out_xy, out_inf);
    std::vector<uint32_t> acc(vk::point_words(ctx->curve));
    VK_TRY(vk::msm_run_host(ctx, t, offset, scalars, n, mont, acc.data()));
    return vk::acc_to_affine(ctx->curve, acc.data(), out_xy, out_inf);
}

int vc_msm_partial(vc_ctx* ctx, int id, size_t offset, const uint64_t* scalars, size_t n, int mont,
                   uint32_t* out_acc) {
    if (!ctx || !out_acc || (n > 0 && !scalars)) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    if (offset > t->n || n > t->n - offset) return VC_E_RANGE;
    return vk::msm_run_host(ctx, t, offset, scalars, n, mont, out_acc);
}

int vc_partials_sum(int curve, const uint32_t* accs, size_t k, uint64_t* out_xy, uint8_t* out_inf) {
    if (!valid_curve(curve) || (k > 0 && !accs) || !out_xy || !out_inf) return VC_E_INVALID;
    std::vector<uint32_t> acc(vk::point_words(curve));
    VK_TRY(vk::acc_sum(curve, accs, k, acc.data()));
    return vk::acc_to_affine(curve, acc.data(), out_xy, out_inf);
}

int vc_fixed_base_precompute(vc_ctx* ctx, int id, int window_bits) {
    if (!ctx) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    return vk::fixed_base_precompute(ctx, t, window_bits);
}

int vc_fixed_base_precompute_windows(vc_ctx* ctx, int id, int window_bits, int windows) {
    if (!ctx || windows < 0) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    return vk::fixed_base_precompute(ctx, t, window_bits, windows);
}

int vc_fixed_base_table_bytes(vc_ctx* ctx, int id, size_t* bytes) {
    if (!ctx || !bytes) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    *bytes = (t->fb_c != 0 && t->fb.p) ? t->fb.cap : 0;
    return VC_OK;
}

int vc_fixed_base_geometry(vc_ctx* ctx, int id, int* window_bits, int* windows, int* wide_windows) {
    if (!ctx) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    const bool built = t->fb_c != 0 && t->fb.p;
    if (window_bits) *window_bits = built ? t->fb_c : 0;
    if (windows) *windows = built ? t->fb_W : 0;
    if (wide_windows) *wide_windows = built ? t->fb_big : 0;
    return VC_OK;
}

int vc_msm_batch_device(vc_ctx* ctx, int id, size_t width, const void* d_sc, size_t batch, int mont,
                        void* d_out_xy, uint8_t* d_out_inf) {
    if (!ctx || (batch > 0 && (!d_sc || !d_out_xy || !d_out_inf)) || width == 0) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    VK_TRY(vk::msm_batch_run(ctx, t, width, d_sc, batch, mont, d_out_xy, d_out_inf));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}

int vc_msm_batch_sparse(vc_ctx* ctx, int id, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                        const uint64_t* scalars, int mont, uint64_t* out_xy, uint8_t* out_inf) {
    if (!ctx || (batch > 0 && (!row_ptr || !out_xy || !out_inf))) return VC_E_INVALID;
    if (batch > 0 && row_ptr[batch] > 0 && (!cols || !scalars)) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    return vk::msm_batch_sparse(ctx, t, batch, row_ptr, cols, scalars, mont, out_xy, out_inf);
}

}  // extern "C"

namespace vk {
int msm_batch_sparse_items_guarded(vc_ctx* ctx, int id, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                                   const uint64_t* scalars, uint64_t* out_xy, uint8_t* out_inf, uint64_t* out_items) {
    if (!ctx || (batch > 0 && (!row_ptr || !out_xy || !out_inf || !out_items))) return VC_E_INVALID;
    if (batch > 0 && row_ptr[batch] > 0 && (!cols || !scalars)) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    return vk::msm_batch_sparse_items(ctx, t, batch, row_ptr, cols, scalars, 0, out_xy, out_inf, out_items);
}
}  // namespace vk

extern "C" {

int vc_msm_batch(vc_ctx* ctx, int id, size_t width, const uint64_t* scalars, size_t batch, int mont,
                 uint64_t* out_xy, uint8_t* out_inf) {
    if (!ctx || (batch > 0 && (!scalars || !out_xy || !out_inf)) || width == 0) return VC_E_INVALID;
    Guard g(ctx);
    vk::Table* t = ctx->table(id);
    if (!t) return VC_E_TABLE;
    return batch_commit_host(ctx, t, width, scalars, batch, mont, out_xy, out_inf);
}

}  // extern "C"
