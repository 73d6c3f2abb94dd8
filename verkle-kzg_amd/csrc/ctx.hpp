// Engine context: one device, one stream, base tables, grow-only workspaces, kernel timers.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/vc_msm.h"

#define VK_CHECK_HIP(expr)                              \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) {                         \
            vk::last_hip_error() = e_;                  \
            return e_ == hipErrorOutOfMemory ? VC_E_OOM : VC_E_HIP; \
        }                                               \
    } while (0)

#define VK_TRY(expr)            \
    do {                        \
        int s_ = (expr);        \
        if (s_ != VC_OK) return s_; \
    } while (0)

namespace vk {

hipError_t& last_hip_error();
int pool_take(vc_ctx* ctx, size_t bytes, void** p, size_t* cap);
void pool_put(vc_ctx* ctx, void* p, size_t cap);
// the live-context registry (capi.cpp) and a block returned to the pool of context `uid` if it
// still exists and its lock is free (else hipFree on device `dev`)
void ctx_register(vc_ctx* ctx, bool live);
void pool_return_uid(uint64_t uid, int dev, void* p, size_t cap);

// hipSetDevice(dev) for a scope, the thread's previous current device restored at its end (helpers
// that touch another context's memory must not leave the caller allocating on that device)
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (dev >= 0 && hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
        else prev = -1;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

// Device buffer. DevBuf(ctx) draws from / returns to the context's stream-ordered block pool
// (per-call scratch of the scheme paths: a hipMalloc + hipFree pair per buffer per call cost
// tens of us each, and hipFree synchronises the device); DevBuf() owns its memory outright.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    vc_ctx* pool = nullptr;
    int ensure(size_t bytes);
    void release();
    explicit DevBuf(vc_ctx* ctx) : pool(ctx) {}
    template <class T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
    ~DevBuf() { release(); }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
};

// page-locked host staging (one per lane): device->host copies into pageable memory go through a
// bounce buffer and start late (measured ~25 us before the MSM's second small read-back)
// compacted rows of the batched commit's latency path (the IPA rounds' L / R): item i < n_main of
// commit g is table base (i / half) m + (g odd ? off_odd : off_even) + i % half, item n_main is
// base `extra` (half = 0: plain rows, item i is base i)
struct StrideCols {
    uint32_t half = 0, m = 0, off_even = 0, off_odd = 0, n_main = 0, extra = 0;
    __host__ __device__ uint32_t base(uint32_t g, uint32_t i) const {
        return i < n_main ? (i / half) * m + ((g & 1) ? off_odd : off_even) + i % half : extra;
    }
};

// The IPA prover's L / R rows made inside the latency-path commit (commit.hip k_fb_commit_small)
// instead of on the host: commit g (proof p = g / 2, L even, R odd), item i < n_main is
// a[p][i % m - h] * coeff[i] for L when i % m >= h, a[p][i % m + h] * coeff[i] for R when i % m < h,
// zero otherwise; item n_main is q[g] (the q' <a, b> term). coeff is this round's coefficient row:
// coeff_in[p] folded by the previous round's challenge x[p] where (i % m_prev) < h_prev (fold != 0),
// written to coeff_out[p] by L's window-0 threads. Montgomery BN254 Fr, 8 words each; a, x and q
// in page-locked host memory (the host folds a and b), coeff in device memory (ping-pong).
struct IpaRows {
    const uint32_t* a = nullptr;  // [B][N] (a_stride = N entries per proof)
    const uint32_t* coeff_in = nullptr;
    uint32_t* coeff_out = nullptr;
    const uint32_t* x = nullptr;  // [B]
    const uint32_t* q = nullptr;  // [2B]
    uint32_t N = 0, m = 0, h = 0, fold = 0, m_prev = 0, h_prev = 0;
};

struct PinBuf {
    void* p = nullptr;
    void* dp = nullptr;     // the device's address of p (kernels read / write it over PCIe)
    size_t cap = 0;
    unsigned flags = 0;     // hipHostMalloc flags (0 = default; hipHostMallocCoherent: fine-grained)
    int ensure(size_t bytes);
    void release();
    template <class T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
    ~PinBuf() { release(); }
    PinBuf() = default;
    PinBuf(const PinBuf&) = delete;
    PinBuf& operator=(const PinBuf&) = delete;
};

// window schedule of a fixed-base table (commit.hip): W signed-digit windows, the last `big` of
// them c + 1 bits wide and the rest c, so a scalar of B bits needs c W + big >= B + 1. Base i's
// block holds stride() entries; window w's 2^(width(w) - 1) multiples start at off(w). Mixed
// widths put a table between two uniform sizes: Bandersnatch c = 18, W = 14, big = 2 is 58 GB
// with the 14 windows of the 101 GB c = 19 table (15 at c = 18).
struct FbGeom {
    int c, W, big;
    __host__ __device__ __forceinline__ int width(int w) const { return c + (w >= W - big ? 1 : 0); }
    __host__ __device__ __forceinline__ size_t off(int w) const {
        return (size_t)(w + (w > W - big ? w - (W - big) : 0)) << (c - 1);
    }
    __host__ __device__ __forceinline__ size_t stride() const { return (size_t)(W + big) << (c - 1); }
};

struct Table {
    int curve = 0;
    size_t n = 0;
    DevBuf bases;  // n x Aff (Montgomery)
    DevBuf inf;    // n x u8
    // fixed-base window tables for batched commits
    int fb_c = 0, fb_W = 0, fb_big = 0;
    bool fb_auto = false;  // built on first use by a commit (counts against the context's budget)
    DevBuf fb;
    FbGeom fb_geom() const { return FbGeom{fb_c, fb_W, fb_big}; }
    // 1: every base lies in the prime-order subgroup (the GLV endomorphism acts as lambda, so
    // msm.hip may split scalars), 0: some base does not, -1: not checked yet
    int subgroup = -1;
    // packed-29 copies (ec29.hpp) read by the accumulate: the bases at [0, n) and, once a GLV
    // MSM has run, phi(P) = (beta x, y) of every base at [n, 2n); built on first use
    int fast_ok = 0, phi_ok = 0;
    DevBuf fast;
    // GLV MSMs over the whole table: packed-29 copies of 2^(c w) P and 2^(c w) phi(P) for every
    // window w ([w][2n] layout), so all windows share one set of buckets (msm.hip, "shared
    // windows"); built on first use for the window size c in win_c
    int win_ok = 0, win_c = 0, win_W = 0, win_ts = 0, win_m = 1;  // win_m > 1: radix win_m 2^win_c
    int win_limbs = 1;  // copies in radix-2^29 limbs (1) or packed-29 (0, VKZG_WIN_PACKED probe)
    int win_pair = 0;   // radix copies in the pair layout (SW29::AffP, one 128-B record per signed copy)
    DevBuf win;
    // the first few bases as a table of their own with wider fixed-base windows (lead_table in
    // commit.hip: the verkle extension rows [1, stem, c1, c2] use bases 0..3 only); owned, built on
    // first use, dropped when the bases are refilled
    Table* lead = nullptr;
    int lead_k = 0, lead_c = 0;
    Table() = default;
    Table(const Table&) = delete;
    Table& operator=(const Table&) = delete;
    ~Table() { delete lead; }
};

enum WsSlot {
    WS_DIGITS = 0,
    WS_COUNTS,
    WS_OFFSETS,
    WS_CURSOR,
    WS_SORTED,
    WS_BUCKETS,
    WS_CARRY,
    WS_THROUGH,
    WS_OWNER,
    WS_OWNER_B,
    WS_SEG,
    WS_WIN,
    WS_SCAN_TMP,
    WS_SCALARS,
    WS_OUT,
    WS_MISC,
    WS_TREE,
    WS_TAIL,
    WS_PIECE,
    WS_SP_RP,
    WS_SP_COLS,
    WS_SP_SC,
    WS_SP_CNT,
    WS_SP_EOFF,
    WS_SP_OFF,
    WS_SP_ROWS,
    WS_SP_XY,
    WS_SP_INF,
    WS_SP_RC,
    WS_SP_CHUNKS,
    WS_CARRY2,
    WS_NXT,
    WS_NXT2,
    WS_CHAIN,
    WS_GLV_SC,
    WS_GLV_FLAG,
    WS_RAW_B,  // radix-29 row sums of the sparse accumulate (converted by k_fast_store)
    WS_SP_ITEMS,  // to_data_item of the sparse commits' rows (msm_batch_sparse_items)
    WS_NORM_CNT,  // the verkle normalisation's arrival counter (zero between launches)
    WS_NORM_TOT,  // its block products and per-block cofactors (device scan)
    WS_COUNT_
};

// a stream and the workspace its launches use: the MSM runs two window slices concurrently
// (lane 0 = the context's stream + ws, lane 1 = side_stream + ws2)
struct Lane {
    hipStream_t st;
    DevBuf* ws;
    PinBuf* pin;
};

struct PendingTimer {
    hipEvent_t a, b;
    std::string name;
};

}  // namespace vk

struct vc_ctx {
    int curve = 0;
    int device = 0;
    uint64_t uid = 0;  // unique per context ever created (a freed context's address can come back)
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    hipStream_t side_stream = nullptr;  // second queue for latency-bound tails
    // recursive: pool_return_uid try_locks the context a released verkle mirror belongs to, and
    // the releasing thread may already own that lock (try_lock by the owner of a plain std::mutex
    // is undefined; on a recursive one it succeeds)
    std::recursive_mutex mu;
    std::vector<vk::Table*> tables;
    vk::DevBuf ws[vk::WS_COUNT_];
    vk::DevBuf ws2[vk::WS_COUNT_];  // workspace of lane 1 (side_stream)
    vk::PinBuf pin[2];              // read-back staging of lanes 0 / 1
    vk::PinBuf pin_io;              // host <-> device staging of the scheme paths (commit_batch)
    vk::PinBuf pin_small;           // block partials of the small-batch commit path (fine-grained:
                                    // the kernel writes them straight to host memory)
    vk::PinBuf pin_norm;            // block products / inverses of the split normalisation
    vk::PinBuf pin_y;               // the KZG opening's y, copied back asynchronously
    vk::PinBuf pin_mp;              // the multiproof finish's h - g, copied back ahead of the E commit
    vk::PinBuf pin_ipa;             // the IPA prover's a, x and q terms read by the round kernel (IpaRows)
    vk::PinBuf pin_verkle;          // the verkle extension rows, merged straight into page-locked memory
    vk::PinBuf pin_verkle2;         // the second buffer of the rows built in pieces (odd pieces)
    vk::PinBuf pin_verkle_lv[2];    // verkle levels' lists (one upload per level; the next level's are
                                    // built into the other one while the current level runs)
    vk::PinBuf pin_norm_vk;         // block products / inverses of the verkle rows' normalisation
    vk::PinBuf pin_sparse_ck;       // chunk tables of the sparse commits' latency path
    vk::PinBuf pin_sparse_ch;       // chunk lists of the sort-based sparse commits
    // free blocks of DevBuf(ctx) scratch (size -> pointer); all their users run on `stream`
    // (or are synchronised), so a block freed by one call is safely reused by the next in
    // stream order; vc_ctx_set_stream drains the old stream first
    std::multimap<size_t, void*> pool_free;
    size_t pool_bytes = 0;
    bool timing = false;
    // vc_ctx_set_option knobs (include/vc_msm.h VC_OPT_*)
    int opt_shared_windows = 1;           // GLV MSMs over a whole table: one bucket set via Table::win
    size_t opt_msm_chunk = size_t(1) << 27;  // MSMs above this many points run as summed chunks
    int opt_host_chunks = 2;                 // vc_msm: scalar copies in this many chunks (msm_run_host)
    uint32_t fb_lanes = 0;                // resident lanes of k_fb_commit_cm (cached per context)
    uint32_t small_epoch = 0;             // completion-flag epoch of the latency path's launches
    uint32_t tail_epoch = 0;              // the same for the MSM tails' direct completion (pin[0 / 1])
    uint32_t norm_vk_parity = 0;          // the half of pin_norm_vk the last verkle normalisation used
    // geometry of the last MSM (vc_msm_last_plan): window bits c, windows W (of the whole MSM),
    // terms per point (2 with the GLV split), radix multiplier m (radix m 2^c; 1 = 2^c), shared
    struct {
        int c, W, terms, m, shared;
    } plan = {0, 0, 0, 0, 0};
    std::vector<vk::PendingTimer> pending;
    std::vector<hipEvent_t> event_pool;
    std::map<std::string, std::pair<double, long>> ktime;
    // effective shader clock of timed accumulate launches: with timing on, the first lane of the
    // grid stamps s_memtime (shader cycles) and s_memrealtime (100 MHz) around its loop into a slot
    // of `clk` (4 u64); collect_timers adds the deltas (vc_ctx_accumulate_clock)
    vk::DevBuf clk;
    std::vector<uint32_t> clk_pending;  // slots written by launches not yet collected
    uint32_t clk_next = 0;
    double clk_cycles = 0.0, clk_ticks = 0.0;
    long clk_n = 0;
    uint64_t* clk_slot();  // nullptr unless timing (and the buffer exists)
    vk::Table scratch;  // variable-base points of verifiers (grow-only)
    // per-domain constant tables (domain powers, 1/(w^k - 1)), keyed by field and size
    std::map<std::string, std::unique_ptr<vk::DevBuf>> dcache;

    hipEvent_t get_event();
    void timer_begin(const char* name, hipEvent_t* a, hipStream_t s = nullptr);
    void timer_end(const char* name, hipEvent_t a, hipStream_t s = nullptr);
    void collect_timers();  // call after the stream is synchronised
    vk::Lane lane(int i) { return i == 0 ? vk::Lane{stream, ws, &pin[0]} : vk::Lane{side_stream, ws2, &pin[1]}; }
    // bytes of the fixed-base tables built on first use that this context still holds (commit.hip
    // fb_default_c's budget; a table refilled or re-precomputed explicitly stops counting)
    size_t fb_auto_used() const {
        size_t s = 0;
        for (const vk::Table* t : tables) {
            if (t && t->fb_auto && t->fb.p) s += t->fb.cap;
            if (t && t->lead && t->lead->fb.p) s += t->lead->fb.cap;  // (built on first use too)
        }
        return s;
    }
    vk::Table* table(int id) {
        if (id < 0 || id >= (int)tables.size() || !tables[id]) return nullptr;
        return tables[id];
    }
};

// launch helper: records HIP events around the launch when timing is on
#define VK_LAUNCH(ctx, name, kernel, grid, block, shmem, ...)                          \
    do {                                                                             \
        hipEvent_t ev_a_ = nullptr;                                                  \
        if ((ctx)->timing) (ctx)->timer_begin(name, &ev_a_);                         \
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), shmem, (ctx)->stream, __VA_ARGS__); \
        if ((ctx)->timing) (ctx)->timer_end(name, ev_a_);                            \
        VK_CHECK_HIP(hipGetLastError());                                             \
    } while (0)

#define VK_LAUNCH_ON(ctx, strm, name, kernel, grid, block, shmem, ...)                 \
    do {                                                                             \
        hipEvent_t ev_a_ = nullptr;                                                  \
        if ((ctx)->timing) (ctx)->timer_begin(name, &ev_a_, strm);                   \
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), shmem, strm, __VA_ARGS__); \
        if ((ctx)->timing) (ctx)->timer_end(name, ev_a_, strm);                      \
        VK_CHECK_HIP(hipGetLastError());                                             \
    } while (0)

namespace vk {
// implemented per translation unit with explicit instantiations
int device_mad_rate(vc_ctx* ctx, double* tera_per_s);
int msm_windows(int curve, size_t n, int* c, int* W, int* terms);
// vc_msm: scalars in host memory (chunked copies under the previous chunk's kernels where the
// geometry allows, msm.hip msm_run_host_chunks_t)
int msm_run_host(vc_ctx* ctx, Table* t, size_t offset, const uint64_t* host_sc, size_t n, int mont, uint32_t* out_acc);
int msm_run(vc_ctx* ctx, Table* t, size_t offset, const void* d_scalars, size_t n, int mont,
            uint32_t* out_acc, int part = 0, int parts = 1);
// K MSMs over the whole table t (scalar set k at d_scalars[k], Montgomery flag mont[k]) -> K
// accumulators; one batched pipeline where the geometry allows (msm.hip msm_run_many_t)
int msm_run_many(vc_ctx* ctx, Table* t, const void* const* d_scalars, const int* mont, size_t n, size_t K,
                 uint32_t* out_accs);
int acc_to_affine(int curve, const uint32_t* acc, uint64_t* out_xy, uint8_t* out_inf);
// n accumulators with one field inversion (Montgomery's trick); same outputs as acc_to_affine
int acc_to_affine_batch(int curve, const uint32_t* accs, size_t n, uint64_t* out_xy, uint8_t* out_inf);
int acc_sum(int curve, const uint32_t* accs, size_t k, uint32_t* out);
int point_words(int curve);
int aff_limbs64(int curve);  // NL of the base field in u64 limbs
int bases_upload(vc_ctx* ctx, const uint64_t* xy, const uint8_t* inf, size_t n, int* id);
int bases_fill(vc_ctx* ctx, Table* t, const uint64_t* xy, const uint8_t* inf, size_t n);
int bases_random(vc_ctx* ctx, uint64_t seed, size_t n, int* id);
int bases_download(vc_ctx* ctx, Table* t, uint64_t* xy, uint8_t* inf);
int fixed_base_precompute(vc_ctx* ctx, Table* t, int c, int windows = 0);
// t's first k bases as their own table with c-bit fixed-base windows (t->lead, built on first
// use); *out = nullptr when it cannot be had (out of memory: the caller keeps t)
int lead_table(vc_ctx* ctx, Table* t, int k, int c, Table** out);
int normalize_to_canon(vc_ctx* ctx, int curve, const void* d_acc, size_t n, void* d_out_xy, uint8_t* d_out_inf);
int msm_batch_sparse(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                     const uint64_t* scalars, int mont, uint64_t* out_xy, uint8_t* out_inf);
// the same with the rows' to_data_item values too (BN254; lib.rs:56-67), computed on the device from
// the normalised points and read back with them (the verkle levels: no second round trip)
int msm_batch_sparse_items(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                           const uint64_t* scalars, int mont, uint64_t* out_xy, uint8_t* out_inf, uint64_t* out_items);
// the same behind the ctx lock, by table id (what vc_msm_batch_sparse does for the plain call)
int msm_batch_sparse_items_guarded(vc_ctx* ctx, int table, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                                   const uint64_t* scalars, uint64_t* out_xy, uint8_t* out_inf, uint64_t* out_items);
// the same on the device (BN254): CSR columns / canonical scalars already in device memory, the row
// structure row_ptr on the host (rows_fit: every row has 1..4 non-zeros -- the chunks are the rows);
// affine rows, flags and items written to device memory, enqueued on ctx->stream (verkle.cpp's
// device-resident levels)
// the sparse commits' latency path (msm.hip k_fb_sparse_small, BN254): rows of (column, scalar)
// non-zeros; mode 0: d_vals (4 canonical words per non-zero), 1: d_vals of 2 words (16-byte
// values), 2: d_item[d_child[j]] - (d_sidx && d_sidx[j] >= 0 ? d_snap[d_sidx[j]] : 0). Row g
// also adds the point (d_add_xy, d_add_inf)[d_add_ids[g]] if given (0xffffffff: none); its
// canonical affine point, identity flag and to_data_item go to index d_dst[g] (null: g) of the
// outputs. Enqueued on ctx->stream; one host round trip (the normalisation), no final sync.
struct SmallRows {
    size_t batch = 0;
    const uint64_t* row_ptr = nullptr;  // host, batch + 1
    int mode = 0;
    const uint32_t* d_cols = nullptr;
    const uint64_t* d_vals = nullptr;
    const uint64_t* d_item = nullptr;
    const uint32_t* d_child = nullptr;
    const int32_t* d_sidx = nullptr;
    const uint64_t* d_snap = nullptr;
    const uint32_t* d_add_ids = nullptr;
    const uint64_t* d_add_xy = nullptr;
    const uint8_t* d_add_inf = nullptr;
    const uint32_t* d_dst = nullptr;
    uint64_t* d_out_xy = nullptr;
    uint8_t* d_out_inf = nullptr;
    uint64_t* d_out_item = nullptr;
};
// overlap (optional): host work run once the kernels and the read-back are queued, before the wait
int sparse_small_items_dev(vc_ctx* ctx, Table* t, const SmallRows& in,
                           const std::function<void()>* overlap = nullptr);
size_t sparse_small_pairs(const Table* t, size_t nnz);  // (non-zero, window) pairs of nnz non-zeros
// BN254 rows -> (optional old-commitment adds) canonical affine points, flags, to_data_item at
// dst[j] (commit.hip); no final sync
int normalize_rows_items(vc_ctx* ctx, void* d_rows, size_t n, const uint32_t* add_ids, const uint64_t* add_xy,
                         const uint8_t* add_inf, const uint32_t* dst, uint64_t* out_xy, uint8_t* out_inf,
                         uint64_t* out_item, const std::function<void()>* overlap = nullptr);
// d_add_ids (optional): row g also adds the canonical affine point (d_add_xy, d_add_inf)[d_add_ids[g]]
// before the normalisation (0xffffffff: nothing) -- a verkle row that updates its old commitment.
// d_dst (optional): row g's outputs go to index d_dst[g] (the tree's mirror). d_row_ptr (optional,
// rows_fit only): a device copy of row_ptr the caller already has (no upload). The normalisation is
// normalize_rows_items' (polled, no stream wait; `overlap` runs once every kernel is queued).
int sparse_commit_items_dev(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, bool rows_fit,
                            const uint32_t* d_cols, const void* d_sc, void* d_xy, uint8_t* d_inf, void* d_items,
                            const uint32_t* d_add_ids = nullptr, const uint64_t* d_add_xy = nullptr,
                            const uint8_t* d_add_inf = nullptr, const uint32_t* d_dst = nullptr,
                            const std::function<void()>* overlap = nullptr, const uint64_t* d_row_ptr = nullptr);
// k_to_data_item over device points (canonical affine u64 x 8 + flags) into device items, on the
// ctx stream (scheme.hip)
int to_data_item_device(vc_ctx* ctx, const void* d_xy, const uint8_t* d_inf, size_t n, void* d_items);
int table_from_acc(vc_ctx* ctx, Table* t, const void* d_acc, size_t n);
// h_out_xy / h_out_inf (optional): host destinations -- when the small-batch latency path ran,
// the results are written there instead of d_out_* and *on_host is set
// pin_sc: the scalars in ctx->pin_io (host, page-locked) instead of d_scalars (nullptr): uploaded
// to WS_SCALARS here, or read in place over PCIe by the latency path. overlap: host work run once
// the commit kernel is enqueued, before the call waits for it. cols: compacted rows (latency path
// only: VC_E_INVALID otherwise; fb_small_path says whether it runs)
int msm_batch_run(vc_ctx* ctx, Table* t, size_t width, const void* d_scalars, size_t batch,
                  int mont, void* d_out_xy, uint8_t* d_out_inf, uint64_t* h_out_xy = nullptr,
                  uint8_t* h_out_inf = nullptr, bool* on_host = nullptr, const PinBuf* pin_sc = nullptr,
                  const std::function<void()>* overlap = nullptr, const StrideCols* cols = nullptr,
                  const IpaRows* ipa = nullptr);
// whether msm_batch_run of `batch` width-`width` commits takes the latency path
bool fb_small_path(vc_ctx* ctx, Table* t, size_t width, size_t batch);
}  // namespace vk
