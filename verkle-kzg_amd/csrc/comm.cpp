// Multi-GPU entry points (include/vc_comm.h): a vc_comm is one rank of a group with an
// all-gather -- RCCL over xGMI (loaded at run time) or a caller-supplied host callback -- and
// the sharded workloads run this rank's share on its vc_ctx, then ONE all-gather per exchange
// step. The reference is single-process CPU code (utils.rs:16-19 and its
// callers), so these have no reference counterpart beyond the per-rank work they split.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/vc_comm.h"
#include "comm.hpp"
#include "scheme_internal.hpp"
#include "ctx.hpp"

namespace {

// RCCL entry points, resolved once with dlopen: the library stays optional (a host-callback
// comm and every single-GPU call work without it), and a process that already loaded torch's
// bundled RCCL does not get a second copy linked in at load time.
struct Rccl {
    bool ok = false;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
        void* h = nullptr;
        for (const char* n : names)
            if ((h = dlopen(n, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
        if (!h) return;
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(h, "ncclCommInitRank"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
        r.ok = r.get_unique_id && r.init_rank && r.all_gather && r.destroy;
    });
    return r;
}

// grow-only device buffer of a comm (its own device, not a ctx pool: the comm outlives calls)
struct Stage {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return VC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
        if (e != hipSuccess) {
            vk::last_hip_error() = e;
            p = nullptr;
            return VC_E_OOM;
        }
        cap = bytes ? bytes : 16;
        return VC_OK;
    }
    ~Stage() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

struct vc_comm {
    int rank = 0, world = 1, device = -1;
    int msm_split = VC_COMM_SPLIT_WINDOWS;  // vc_comm_set_msm_split
    ncclComm_t nccl = nullptr;
    vc_allgather_fn fn = nullptr;
    void* user = nullptr;
    Stage send, recv, work;  // RCCL staging of host buffers; sharded-workload scratch
    std::vector<uint8_t> hbuf;  // host staging of device all-gathers over a callback comm
};

namespace {

int comm_allgather_dev(vc_comm* c, vc_ctx* ctx, const void* d_send, size_t bytes, void* d_recv);

// RCCL staging of host exchanges: fixed pieces through buffers allocated once at init, so an
// exchange never allocates (a rank that failed to grow a buffer could not enter the collective)
constexpr size_t HOST_PIECE = size_t(1) << 20;

// host buffers -> host buffers
int comm_allgather_host(vc_comm* c, vc_ctx* ctx, const void* send, size_t bytes, void* recv) {
    if (!c->nccl && c->world == 1) {
        if (bytes && recv != send) memcpy(recv, send, bytes);
        return VC_OK;
    }
    if (!c->nccl) return c->fn(c->user, send, bytes, recv) == 0 ? VC_OK : VC_E_COMM;
    if (!ctx) return VC_E_INVALID;
    (void)hipSetDevice(ctx->device);
    const uint8_t* s = static_cast<const uint8_t*>(send);
    uint8_t* r = static_cast<uint8_t*>(recv);
    for (size_t off = 0; off < bytes; off += HOST_PIECE) {  // same piece sequence on every rank
        const size_t m = std::min(HOST_PIECE, bytes - off);
        VK_CHECK_HIP(hipMemcpyAsync(c->send.p, s + off, m, hipMemcpyHostToDevice, ctx->stream));
        VK_TRY(comm_allgather_dev(c, ctx, c->send.p, m, c->recv.p));
        for (int k = 0; k < c->world; k++)
            VK_CHECK_HIP(hipMemcpyAsync(r + (size_t)k * bytes + off, static_cast<uint8_t*>(c->recv.p) + (size_t)k * m, m,
                                        hipMemcpyDeviceToHost, ctx->stream));
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return VC_OK;
}

// the group's statuses of one step (a 4-byte exchange): every rank learns whether all shares
// succeeded. Returns own status if it failed, VC_E_PEER if only a peer failed, else VC_OK (or
// the exchange's own error).
int agree(vc_comm* c, vc_ctx* ctx, int st) {
    std::vector<int32_t> all(c->world);
    const int32_t mine = st;
    const int cs = comm_allgather_host(c, ctx, &mine, 4, all.data());
    if (cs != VC_OK) return cs;
    if (st != VC_OK) return st;
    for (int k = 0; k < c->world; k++)
        if (all[k] != VC_OK) return VC_E_PEER;
    return VC_OK;
}
// the same for statuses already gathered inside the records (stride bytes apart, status first)
int agree_in(const vc_comm* c, int st, const uint8_t* recs, size_t stride) {
    if (st != VC_OK) return st;
    for (int k = 0; k < c->world; k++) {
        int32_t v;
        memcpy(&v, recs + (size_t)k * stride, 4);
        if (v != VC_OK) return VC_E_PEER;
    }
    return VC_OK;
}

// device buffers (ctx's device) -> device buffers; synchronous
int comm_allgather_dev(vc_comm* c, vc_ctx* ctx, const void* d_send, size_t bytes, void* d_recv) {
    (void)hipSetDevice(ctx->device);
    if (c->nccl) {
        if (rccl().all_gather(d_send, d_recv, bytes, ncclUint8, c->nccl, ctx->stream) != ncclSuccess)
            return VC_E_COMM;
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        return VC_OK;
    }
    if (c->world == 1) {
        VK_CHECK_HIP(hipMemcpyAsync(d_recv, d_send, bytes, hipMemcpyDeviceToDevice, ctx->stream));
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        return VC_OK;
    }
    c->hbuf.resize(bytes * (c->world + 1));
    uint8_t* hs = c->hbuf.data();
    uint8_t* hr = hs + bytes;
    VK_CHECK_HIP(hipMemcpyAsync(hs, d_send, bytes, hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    if (c->fn(c->user, hs, bytes, hr) != 0) return VC_E_COMM;
    VK_CHECK_HIP(hipMemcpyAsync(d_recv, hr, bytes * c->world, hipMemcpyHostToDevice, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}

// one exchange of projective partials: record = status word + the partial (zero on failure);
// every rank sums the partials or returns the group's error
template <class Fn>
int partial_step(vc_ctx* ctx, vc_comm* comm, Fn&& compute, uint64_t* out_xy, uint8_t* out_inf) {
    const int words = vk::point_words(ctx->curve);
    const size_t rec = (size_t)words + 1;
    std::vector<uint32_t> part(rec, 0), parts(rec * comm->world);
    const int st = compute(part.data() + 1);
    if (st != VC_OK) std::fill(part.begin(), part.end(), 0u);
    part[0] = (uint32_t)st;
    VK_TRY(comm_allgather_host(comm, ctx, part.data(), rec * 4, parts.data()));
    VK_TRY(agree_in(comm, st, reinterpret_cast<const uint8_t*>(parts.data()), rec * 4));
    std::vector<uint32_t> acc((size_t)words * comm->world);
    for (int k = 0; k < comm->world; k++) memcpy(&acc[(size_t)k * words], &parts[k * rec + 1], (size_t)words * 4);
    return vc_partials_sum(ctx->curve, acc.data(), comm->world, out_xy, out_inf);
}

bool valid(const vc_comm* c, const vc_ctx* ctx) { return c && ctx && (!c->nccl || c->device == ctx->device); }

}  // namespace

extern "C" {

int vc_comm_unique_id(uint8_t id[VC_COMM_ID_BYTES]) {
    if (!id) return VC_E_INVALID;
    const Rccl& r = rccl();
    if (!r.ok) return VC_E_NO_DEVICE;
    ncclUniqueId u;
    if (r.get_unique_id(&u) != ncclSuccess) return VC_E_COMM;
    static_assert(sizeof(u) == VC_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, VC_COMM_ID_BYTES);
    return VC_OK;
}

int vc_comm_init_rccl(int device, int rank, int world, const uint8_t id[VC_COMM_ID_BYTES], vc_comm** out) {
    if (!out || !id || world < 1 || rank < 0 || rank >= world) return VC_E_INVALID;
    *out = nullptr;
    const Rccl& r = rccl();
    if (!r.ok) return VC_E_NO_DEVICE;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return VC_E_NO_DEVICE;
    if (device < 0 || device >= ndev) return VC_E_INVALID;
    VK_CHECK_HIP(hipSetDevice(device));
    ncclUniqueId u;
    memcpy(&u, id, VC_COMM_ID_BYTES);
    ncclComm_t nc = nullptr;
    if (r.init_rank(&nc, world, u, rank) != ncclSuccess) return VC_E_COMM;
    vc_comm* c = new vc_comm();
    c->rank = rank;
    c->world = world;
    c->device = device;
    c->nccl = nc;
    // host-exchange staging, once (comm_allgather_host moves fixed pieces through it)
    if (c->send.ensure(HOST_PIECE) != VC_OK || c->recv.ensure(HOST_PIECE * world) != VC_OK) {
        vc_comm_destroy(c);
        return VC_E_OOM;
    }
    *out = c;
    return VC_OK;
}

int vc_comm_init_host(int rank, int world, vc_allgather_fn fn, void* user, vc_comm** out) {
    if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !fn)) return VC_E_INVALID;
    vc_comm* c = new vc_comm();
    c->rank = rank;
    c->world = world;
    c->fn = fn;
    c->user = user;
    *out = c;
    return VC_OK;
}

void vc_comm_destroy(vc_comm* c) {
    if (!c) return;
    if (c->device >= 0) (void)hipSetDevice(c->device);
    if (c->nccl) (void)rccl().destroy(c->nccl);
    delete c;
}

int vc_comm_rank(const vc_comm* c) { return c ? c->rank : VC_E_INVALID; }
int vc_comm_world(const vc_comm* c) { return c ? c->world : VC_E_INVALID; }
int vc_comm_is_rccl(const vc_comm* c) { return c ? (c->nccl != nullptr) : VC_E_INVALID; }

int vc_comm_allgather(vc_comm* c, vc_ctx* ctx, const void* send, size_t bytes, void* recv) {
    if (!c || (bytes && (!send || !recv)) || (c->nccl && !valid(c, ctx))) return VC_E_INVALID;
    return comm_allgather_host(c, ctx, send, bytes, recv);
}

// ---------------------------------------------------------------- sharded workloads



int vc_comm_set_msm_split(vc_comm* c, int split) {
    if (!c || (split != VC_COMM_SPLIT_WINDOWS && split != VC_COMM_SPLIT_POINTS)) return VC_E_INVALID;
    c->msm_split = split;
    return VC_OK;
}

int vc_msm_sharded(vc_ctx* ctx, vc_comm* comm, int table_id, size_t offset, const void* d_scalars, size_t n, int mont,
                   uint64_t* out_xy, uint8_t* out_inf) {
    if (!valid(comm, ctx) || !out_xy || !out_inf) return VC_E_INVALID;
    if (comm->msm_split == VC_COMM_SPLIT_POINTS)
        return partial_step(ctx, comm, [&](uint32_t* part) {
            size_t lo, hi;
            vk::shard_range(n, comm->rank, comm->world, &lo, &hi);
            const uint8_t* sc = static_cast<const uint8_t*>(d_scalars);
            return vc_msm_device_partial(ctx, table_id, offset + lo, sc ? sc + lo * 32 : nullptr, hi - lo, mont, part);
        }, out_xy, out_inf);
    return partial_step(ctx, comm, [&](uint32_t* part) {
        return vc_msm_device_window_part(ctx, table_id, offset, d_scalars, n, mont, comm->rank, comm->world, part);
    }, out_xy, out_inf);
}

int vc_msm_batch_sharded(vc_ctx* ctx, vc_comm* comm, int table_id, size_t width, const void* d_scalars, size_t batch,
                         int mont, uint64_t* out_xy, uint8_t* out_inf) {
    if (!valid(comm, ctx) || width == 0 || (batch && (!d_scalars || !out_xy || !out_inf))) return VC_E_INVALID;
    if (batch == 0) return VC_OK;
    const size_t W2 = 2 * (size_t)vk::aff_limbs64(ctx->curve);  // u64 words of one affine point
    size_t lo, hi;
    vk::shard_range(batch, comm->rank, comm->world, &lo, &hi);
    const size_t bmax = (batch + comm->world - 1) / comm->world, mine = hi - lo;
    const size_t rec = W2 + 1;  // u64 words per record: x, y, inf
    const size_t slot = 1 + bmax * rec;  // a rank's status word, then its records
    std::vector<uint64_t> send(slot, 0), recv(slot * comm->world);
    int st = VC_OK;
    if (mine > 0) {
        auto share = [&]() -> int {
            (void)hipSetDevice(ctx->device);
            VK_TRY(comm->work.ensure(mine * (W2 * 8 + 1)));
            uint8_t* dxy = reinterpret_cast<uint8_t*>(comm->work.p);
            uint8_t* dinf = dxy + mine * W2 * 8;
            const uint8_t* sc = reinterpret_cast<const uint8_t*>(d_scalars) + lo * width * 32;
            VK_TRY(vc_msm_batch_device(ctx, table_id, width, sc, mine, mont, dxy, dinf));
            std::vector<uint64_t> hxy(mine * W2);
            std::vector<uint8_t> hinf(mine);
            VK_CHECK_HIP(hipMemcpy(hxy.data(), dxy, mine * W2 * 8, hipMemcpyDeviceToHost));
            VK_CHECK_HIP(hipMemcpy(hinf.data(), dinf, mine, hipMemcpyDeviceToHost));
            for (size_t b = 0; b < mine; b++) {
                memcpy(&send[1 + b * rec], &hxy[b * W2], W2 * 8);
                send[1 + b * rec + W2] = hinf[b];
            }
            return VC_OK;
        };
        st = share();  // a failed share still enters the exchange (vc_comm.h)
    }
    send[0] = (uint64_t)(uint32_t)st;
    VK_TRY(comm_allgather_host(comm, ctx, send.data(), send.size() * 8, recv.data()));
    VK_TRY(agree_in(comm, st, reinterpret_cast<const uint8_t*>(recv.data()), slot * 8));
    for (int k = 0; k < comm->world; k++) {
        size_t a, e;
        vk::shard_range(batch, k, comm->world, &a, &e);
        const uint64_t* src = &recv[(size_t)k * slot + 1];
        for (size_t b = 0; b < e - a; b++) {
            memcpy(&out_xy[(a + b) * W2], &src[b * rec], W2 * 8);
            out_inf[a + b] = (uint8_t)src[b * rec + W2];
        }
    }
    return VC_OK;
}

int vc_kzg_prove_sharded(vc_ctx* ctx, vc_comm* comm, int table, size_t size, const void* d_evals, size_t max,
                         const uint64_t* point, uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y) {
    if (!valid(comm, ctx) || !point || !proof_xy || !proof_inf || !y) return VC_E_INVALID;
    return partial_step(ctx, comm, [&](uint32_t* part) {
        return vc_kzg_prove_device_part(ctx, table, size, d_evals, max, point, comm->rank, comm->world, part, y);
    }, proof_xy, proof_inf);
}

int vc_multiproof_prove_sharded(vc_ctx* ctx, vc_comm* comm, int scheme, int table, size_t N, size_t Q,
                                const void* d_data_slice, const uint64_t* com_xy, const uint8_t* com_inf,
                                const uint64_t* z, const uint64_t* y, uint64_t* d_xy, uint8_t* d_inf,
                                vc_ipa_proof* ipa_proof, uint64_t* kzg_proof_xy, uint8_t* kzg_proof_inf,
                                uint64_t* kzg_y) {
    if (!valid(comm, ctx) || !com_xy || !com_inf || !z || !y || !d_xy || !d_inf || Q == 0) return VC_E_INVALID;
    if (scheme != 0 && scheme != 1) return VC_E_INVALID;
    vc_transcript* tr = nullptr;
    uint64_t r[4];
    size_t rows = 0;
    size_t lo, hi;
    vk::shard_range(Q, comm->rank, comm->world, &lo, &hi);
    // this rank's share up to the exchange; its status is agreed on before the device all-gather
    // (a rank without its S buffer cannot enter that collective)
    // rows of S = the distinct z (validated here, as the begin call would)
    int st = vk::mp_rows(N, Q, z, &rows);
    const size_t sbytes = rows * N * 32;
    uint8_t* dS = nullptr;
    if (st == VC_OK) {
        (void)hipSetDevice(ctx->device);
        // [0, sbytes): this rank's S; [sbytes, ...): every rank's S in rank order
        st = comm->work.ensure(sbytes * (comm->world + 1));
        if (st == VC_OK) {
            dS = reinterpret_cast<uint8_t*>(comm->work.p);
            // the host transcript overlapped with the shard's plan (scheme.hip mp_begin_accumulate)
            st = vk::mp_begin_accumulate(ctx, N, Q, com_xy, com_inf, z, y, lo, hi - lo, d_data_slice, dS, &tr, r);
        }
    }
    st = agree(comm, ctx, st);
    if (st == VC_OK) st = comm_allgather_dev(comm, ctx, dS, sbytes, dS + sbytes);
    if (st == VC_OK)
        st = vc_multiproof_finish(ctx, scheme, table, N, Q, z, dS + sbytes, comm->world, tr, d_xy, d_inf, ipa_proof,
                                  kzg_proof_xy, kzg_proof_inf, kzg_y);
    if (tr) vc_transcript_free(tr);
    return st;
}

// ---- proof-parallel multiproofs: rank k proves proofs shard_range(P, k, G) end to end
// (vc_multiproof_prove_many), one all-gather of the finished proofs (D, and the IPA proof or the
// KZG (proof, y)) gives every rank all P. The query-sliced single multiproof above cannot go
// much below one GPU's time: every rank repeats the serial host transcript (~2.7 ms at Q = 2^16)
// and the finish (~1.8 ms), so it scales at most ~1.15x on 8 GPUs; independent proofs scale with
// the ranks.
int vc_multiproof_gather(vc_comm* comm, vc_ctx* ctx, int status, int scheme, size_t N, size_t P, uint64_t* d_xy,
                         uint8_t* d_inf, vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy, uint8_t* kzg_inf,
                         uint64_t* kzg_y) {
    // a rank that cannot enter the exchange at all, or group-wide parameters that size the records
    // (every rank of an SPMD call passes the same scheme and N, so all of them return here alike)
    if (!comm || (comm->nccl && !valid(comm, ctx)) || (scheme != 0 && scheme != 1) || N == 0 || (N & (N - 1)))
        return VC_E_INVALID;
    size_t K = 0;
    while ((size_t(1) << K) < N) K++;
    // this rank's output buffers, for all P proofs (it receives every rank's): a bad buffer is this
    // rank's failure, carried in its record like a failed share, so the peers return VC_E_PEER and
    // no rank writes any output before the group has agreed
    int st = status;
    if (st == VC_OK && P && (!d_xy || !d_inf || (scheme == 0 && !ipa_proofs) || (scheme == 1 && (!kzg_xy || !kzg_inf || !kzg_y))))
        st = VC_E_INVALID;
    for (size_t p = 0; st == VC_OK && scheme == 0 && p < P; p++) {
        const vc_ipa_proof& pr = ipa_proofs[p];
        if (pr.rounds < K || (K && (!pr.l_xy || !pr.r_xy || !pr.l_inf || !pr.r_inf)))
            st = VC_E_INVALID;
    }
    const size_t rec = scheme == 0 ? 9 + 18 * K + 8 : 9 + 13;  // u64 words per proof
    size_t lo, hi;
    vk::shard_range(P, comm->rank, comm->world, &lo, &hi);
    const size_t bmax = (P + comm->world - 1) / comm->world, slot = 1 + bmax * rec;
    std::vector<uint64_t> send(slot, 0), recv(slot * comm->world);
    send[0] = (uint64_t)(uint32_t)st;
    for (size_t p = lo; st == VC_OK && p < hi; p++) {
        uint64_t* r = &send[1 + (p - lo) * rec];
        memcpy(r, d_xy + p * 8, 64);
        r[8] = d_inf[p];
        if (scheme == 0) {
            const vc_ipa_proof& pr = ipa_proofs[p];
            for (size_t k = 0; k < K; k++) {
                memcpy(r + 9 + 18 * k, pr.l_xy + 8 * k, 64);
                r[9 + 18 * k + 8] = pr.l_inf[k];
                memcpy(r + 9 + 18 * k + 9, pr.r_xy + 8 * k, 64);
                r[9 + 18 * k + 17] = pr.r_inf[k];
            }
            memcpy(r + 9 + 18 * K, pr.tip, 32);
            memcpy(r + 9 + 18 * K + 4, pr.y, 32);
        } else {
            memcpy(r + 9, kzg_xy + p * 8, 64);
            r[17] = kzg_inf[p];
            memcpy(r + 18, kzg_y + p * 4, 32);
        }
    }
    VK_TRY(comm_allgather_host(comm, ctx, send.data(), send.size() * 8, recv.data()));
    VK_TRY(agree_in(comm, st, reinterpret_cast<const uint8_t*>(recv.data()), slot * 8));
    for (int k = 0; k < comm->world; k++) {
        size_t a, e;
        vk::shard_range(P, k, comm->world, &a, &e);
        for (size_t p = a; p < e; p++) {
            const uint64_t* r = &recv[(size_t)k * slot + 1 + (p - a) * rec];
            memcpy(d_xy + p * 8, r, 64);
            d_inf[p] = (uint8_t)r[8];
            if (scheme == 0) {
                vc_ipa_proof& pr = ipa_proofs[p];
                pr.rounds = K;
                for (size_t j = 0; j < K; j++) {
                    memcpy(pr.l_xy + 8 * j, r + 9 + 18 * j, 64);
                    pr.l_inf[j] = (uint8_t)r[9 + 18 * j + 8];
                    memcpy(pr.r_xy + 8 * j, r + 9 + 18 * j + 9, 64);
                    pr.r_inf[j] = (uint8_t)r[9 + 18 * j + 17];
                }
                memcpy(pr.tip, r + 9 + 18 * K, 32);
                memcpy(pr.y, r + 9 + 18 * K + 4, 32);
            } else {
                memcpy(kzg_xy + p * 8, r + 9, 64);
                kzg_inf[p] = (uint8_t)r[17];
                memcpy(kzg_y + p * 4, r + 18, 32);
            }
        }
    }
    return VC_OK;
}

int vc_multiproof_prove_many_sharded(vc_ctx* ctx, vc_comm* comm, int scheme, int table, size_t N, size_t Q, size_t P,
                                     const void* d_data_mine, const uint64_t* com_xy, const uint8_t* com_inf,
                                     const uint64_t* z, const uint64_t* y, uint64_t* d_xy, uint8_t* d_inf,
                                     vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy, uint8_t* kzg_inf, uint64_t* kzg_y) {
    if (!valid(comm, ctx)) return VC_E_INVALID;
    size_t lo, hi;
    vk::shard_range(P, comm->rank, comm->world, &lo, &hi);
    const int st = hi > lo ? vc_multiproof_prove_many(ctx, scheme, table, N, Q, hi - lo, d_data_mine,
                                                      com_xy ? com_xy + lo * Q * 8 : nullptr,
                                                      com_inf ? com_inf + lo * Q : nullptr, z ? z + lo * Q : nullptr,
                                                      y ? y + lo * Q * 4 : nullptr, d_xy ? d_xy + lo * 8 : nullptr,
                                                      d_inf ? d_inf + lo : nullptr, ipa_proofs ? ipa_proofs + lo : nullptr,
                                                      kzg_xy ? kzg_xy + lo * 8 : nullptr, kzg_inf ? kzg_inf + lo : nullptr,
                                                      kzg_y ? kzg_y + lo * 4 : nullptr)
                           : VC_OK;
    return vc_multiproof_gather(comm, ctx, st, scheme, N, P, d_xy, d_inf, ipa_proofs, kzg_xy, kzg_inf, kzg_y);
}

int vc_verkle_commitment_sharded(vc_ctx* ctx, vc_comm* comm, int table, vc_verkle* tree, uint64_t* out_xy,
                                 uint8_t* out_inf) {
    if (!valid(comm, ctx) || !tree || !out_xy || !out_inf) return VC_E_INVALID;
    vk::Shard sh;
    sh.rank = comm->rank;
    sh.world = comm->world;
    sh.allgather = [&](const void* send, size_t bytes, void* recv) {
        return comm_allgather_host(comm, ctx, send, bytes, recv);
    };
    return vk::verkle_commitment(ctx, table, tree, out_xy, out_inf, &sh);
}

}  // extern "C"
