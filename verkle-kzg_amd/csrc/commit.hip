// Batched fixed-base commits: thousands of width-w commitments against one small CRS
// (IPA::commit ipa/mod.rs:130-135 at N = 256; verkle Node::gen_commitment node.rs:243-271;
// the commit phase of prove_multiproof multiproof.rs:151,168). Config 3 of BASELINE.json.
//
// MI355X-first design: the bases never change, so each base G_i gets a window table
//     T[i][w][k] = (k+1) * 2^(c*w) * G_i     (affine, Montgomery; k < 2^(c-1))
// held in HBM (width 256, c = 8: 67 MB BN254 / 100 MB Bandersnatch -- L3-resident; c = 16:
// 8.6-13 GB, which only a 288 GB part can afford). A commit is then sum over (i, w) of
// +-T[i][w][|d_iw|-1]: W mixed adds per base, no doublings, no buckets. Two schedules:
// throughput (large batches: persistent equal runs of (commit, base) items, one resident
// round, piece combine, workgroup batch inversion) and latency (small batches such as the
// IPA prover's L/R: per-window threads, wave/LDS fold, host combine + normalisation).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "ec.hpp"
#include "ec29.hpp"

namespace vk {

// Table entry: FbE<C> (ec29.hpp).

// copy one window's NBw normalised multiples into the table: tab[i*stride + off(w) + k] =
// aff[i*NBw + k], in the packed-29 form the commit loops read
template <class C>
__global__ void k_fb_place(const typename C::Aff* __restrict__ aff, uint32_t n, uint32_t NBw, FbGeom g, int w,
                           FbE<C>* __restrict__ tab) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (size_t)n * NBw) return;
    size_t i = j / NBw, k = j - i * NBw;
    using FC = typename Fast29<C>::type;
    typename C::Aff packed;
    FC::pack_aff(aff[j], &packed);  // canonical x R'
    tab[i * g.stride() + g.off(w) + k].u = FC::load(&packed);
}

// signed digits of a scalar over the table's windows (widths g.width(w)): d in (-2^(cw-1), 2^(cw-1)]
template <class Fr>
struct FbDigits {
    fe<Fr> s;
    uint32_t carry = 0;
    __device__ __forceinline__ int32_t next(int cw) {
        const uint32_t mask = (1u << cw) - 1, half = 1u << (cw - 1);
        const uint32_t raw = (s.v[0] & mask) + carry;
#pragma unroll
        for (int k = 0; k < 7; k++) s.v[k] = (s.v[k] >> cw) | (s.v[k + 1] << (32 - cw));
        s.v[7] >>= cw;
        carry = raw > half ? 1u : 0u;
        return carry ? (int32_t)raw - (int32_t)(1u << cw) : (int32_t)raw;
    }
};

template <class Fr>
__device__ __forceinline__ fe<Fr> load_scalar_fb(const uint32_t* __restrict__ sc, size_t i) {
    const uint4* p = reinterpret_cast<const uint4*>(sc + 8 * i);
    uint4 a = p[0], b = p[1];
    fe<Fr> s;
    s.v[0] = a.x; s.v[1] = a.y; s.v[2] = a.z; s.v[3] = a.w;
    s.v[4] = b.x; s.v[5] = b.y; s.v[6] = b.z; s.v[7] = b.w;
    return s;
}

template <class C>
__device__ typename C::Acc mul_small_fb(const typename C::Acc& p, uint32_t k) {
    typename C::Acc r = C::zero();
    if (k == 0) return r;
    int top = 31 - __builtin_clz(k);
    r = p;
    for (int i = top - 1; i >= 0; i--) {
        r = C::dbl(r);
        if ((k >> i) & 1) r = C::add(r, p);
    }
    return r;
}

// Q[i] = 2^(c*w) * G_i for the given window (chained: caller passes the previous window)
template <class C>
__global__ void k_fb_shift(typename C::Acc* __restrict__ Q, const typename C::Aff* __restrict__ bases,
                           uint32_t n, int c, int first) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    typename C::Acc q;
    if (first) q = C::from_aff(bases[i], false);
    else {
        q = Q[i];
        for (int k = 0; k < c; k++) q = C::dbl(q);
    }
    Q[i] = q;
}

// tmp[i][k] = (k+1) * Q[i], chunks of CH consecutive k per thread
template <class C>
__global__ void k_fb_fill(const typename C::Acc* __restrict__ Q, uint32_t n, uint32_t NBk, uint32_t CH,
                          typename C::Acc* __restrict__ tmp) {
    uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t nch = (NBk + CH - 1) / CH;
    uint32_t i = gid / nch, ch = gid % nch;
    if (i >= n) return;
    typename C::Acc q = Q[i];
    uint32_t k0 = ch * CH, k1 = min(k0 + CH, NBk);
    typename C::Acc p = mul_small_fb<C>(q, k0 + 1);
    for (uint32_t k = k0; k < k1; k++) {
        tmp[(size_t)i * NBk + k] = p;
        p = C::add(p, q);
    }
}

// ------------------------------------------------------------------ batch normalisation
// One workgroup normalises 256 consecutive accumulators with one field inversion:
// prefix/suffix products by LDS scans, inv_j = inv(prod) * prefix_{j-1} * suffix_{j+1}.
template <class C>
__device__ __forceinline__ fe<typename C::F> denom(const typename C::Acc& a) {
    if constexpr (C::is_te) return a.Z;
    else return a.zzz;
}

// accumulators that take denominator 1 in the batch inversion: the SW identity (Z = 0, nothing
// to invert). An Edwards point always has Z != 0 -- its identity (0 : Z : Z) included, which must
// be divided by Z like any other point (it was counted as 1 and came out as (0, Z), not (0, 1))
template <class C>
__device__ __forceinline__ bool norm_as_one(const typename C::Acc& a) {
    if constexpr (C::is_te) return false;
    else return C::is_zero(a);
}

template <class C>
__global__ void __launch_bounds__(256) k_normalize(const typename C::Acc* __restrict__ in, size_t count,
                                                  typename C::Aff* __restrict__ out_aff,
                                                  uint32_t* __restrict__ out_canon,
                                                  uint8_t* __restrict__ out_inf) {
    using F = typename C::F;
    __shared__ fe<F> pre[256];
    __shared__ fe<F> suf[256];
    size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t tid = threadIdx.x;
    typename C::Acc a = j < count ? in[j] : C::zero();
    bool ident = C::is_zero(a);
    fe<F> z = (j < count && !norm_as_one<C>(a)) ? denom<C>(a) : fe_one<F>();
    pre[tid] = z;
    suf[tid] = z;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {
        fe<F> p = pre[tid], s = suf[tid];
        if (tid >= off) p = fe_mul<F>(pre[tid - off], p);
        if (tid + off < 256) s = fe_mul<F>(s, suf[tid + off]);
        __syncthreads();
        pre[tid] = p;
        suf[tid] = s;
        __syncthreads();
    }
    __shared__ fe<F> tinv;
    if (tid == 0) tinv = fe_inv_bin<F>(pre[255]);
    __syncthreads();
    fe<F> iz = tinv;
    if (tid > 0) iz = fe_mul<F>(iz, pre[tid - 1]);
    if (tid < 255) iz = fe_mul<F>(iz, suf[tid + 1]);
    if (j >= count) return;
    fe<F> x, y;
    if constexpr (C::is_te) {
        x = fe_mul<F>(a.X, iz);
        y = fe_mul<F>(a.Y, iz);
        ident = fe_is_zero<F>(x) && fe_eq<F>(y, fe_one<F>());
    } else {
        fe<F> t = fe_mul<F>(iz, a.zz);  // 1/Z
        x = fe_mul<F>(a.x, fe_sqr<F>(t));
        y = fe_mul<F>(a.y, iz);
    }
    if (out_aff) {
        typename C::Aff r;
        r.x = x;
        r.y = y;
        if constexpr (C::is_te) r.kt = fe_mul<F>(fe_mul<F>(x, y), C::d());
        out_aff[j] = r;
    }
    if (out_canon) {
        fe<F> cx = fe_from_mont<F>(x), cy = fe_from_mont<F>(y);
        if (ident && !C::is_te) {
            cx = fe_zero<F>();
            cy = fe_zero<F>();
        }
#pragma unroll
        for (int k = 0; k < F::N; k++) {
            out_canon[j * 2 * F::N + k] = cx.v[k];
            out_canon[j * 2 * F::N + F::N + k] = cy.v[k];
        }
    }
    if (out_inf) out_inf[j] = ident ? 1 : 0;
}

// Split normalisation: the single field inversion of each 256-element block is what k_normalize
// waits for (~130 us on one GPU lane: a lone wave's serial binary-Euclid loop), while the host
// inverts in a few us. k_norm_prep leaves each element the product of its block's OTHER
// denominators and the block product; the host inverts all block products with one inversion
// (Montgomery's trick) and k_norm_finish scales. One pinned round trip (~20 us) replaces the
// lane inversion: 10k Bandersnatch commits normalise in ~0.06 instead of 0.18 ms.
template <class C>
__device__ __forceinline__ void norm_prep_block(const typename C::Acc& a, size_t j, size_t count,
                                                fe<typename C::F>* __restrict__ others,
                                                fe<typename C::F>* __restrict__ tot) {
    using F = typename C::F;
    __shared__ fe<F> pre[256];
    __shared__ fe<F> suf[256];
    const uint32_t tid = threadIdx.x;
    fe<F> z = (j < count && !norm_as_one<C>(a)) ? denom<C>(a) : fe_one<F>();
    pre[tid] = z;
    suf[tid] = z;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {
        fe<F> p = pre[tid], q = suf[tid];
        if (tid >= off) p = fe_mul<F>(pre[tid - off], p);
        if (tid + off < 256) q = fe_mul<F>(q, suf[tid + off]);
        __syncthreads();
        pre[tid] = p;
        suf[tid] = q;
        __syncthreads();
    }
    fe<F> o = fe_one<F>();
    if (tid > 0) o = pre[tid - 1];
    if (tid < 255) o = tid > 0 ? fe_mul<F>(o, suf[tid + 1]) : suf[tid + 1];
    if (j < count) others[j] = o;
    if (tid == 0) tot[blockIdx.x] = pre[255];
}
template <class C>
__global__ void __launch_bounds__(256) k_norm_prep(const typename C::Acc* __restrict__ in, size_t count,
                                                  fe<typename C::F>* __restrict__ others,
                                                  fe<typename C::F>* __restrict__ tot) {
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    norm_prep_block<C>(j < count ? in[j] : C::zero(), j, count, others, tot);
}
// verkle rows (BN254): row j first takes the canonical affine point (add_xy, add_inf)[add_ids[j]]
// (0xffffffff: none) -- the old commitment of a delta row -- and is written back with it
__global__ void __launch_bounds__(256) k_norm_prep_vk(BN254G1::Acc* __restrict__ rows, size_t count,
                                                     const uint32_t* __restrict__ add_ids,
                                                     const uint64_t* __restrict__ add_xy,
                                                     const uint8_t* __restrict__ add_inf,
                                                     fe<BN254Fq>* __restrict__ others, fe<BN254Fq>* __restrict__ tot,
                                                     uint32_t* __restrict__ flags, uint32_t epoch,
                                                     uint32_t* __restrict__ counter, fe<BN254Fq>* __restrict__ cof,
                                                     fe<BN254Fq>* __restrict__ total, uint64_t* __restrict__ tags) {
    using C = BN254G1;
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    C::Acc a = j < count ? rows[j] : C::zero();
    if (add_ids && j < count) {
        const uint32_t id = add_ids[j];
        if (id != 0xffffffffu && !add_inf[id]) {
            C::Aff q;
            memcpy(q.x.v, add_xy + 8 * (size_t)id, 32);
            memcpy(q.y.v, add_xy + 8 * (size_t)id + 4, 32);
            q.x = fe_to_mont<BN254Fq>(q.x);
            q.y = fe_to_mont<BN254Fq>(q.y);
            a = C::madd(a, q, false);
            rows[j] = a;
        }
    }
    norm_prep_block<C>(a, j, count, others, tot);
    if (counter == nullptr) {
        // tot in fine-grained host memory (normalize_rows_items): the block product is made visible
        // system wide, then the block's flag takes this launch's epoch (the host polls the flags)
        if (flags != nullptr && threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(&flags[blockIdx.x], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    // device scan (tot in device memory): the last block to arrive turns the nblk block products
    // into per-block cofactors cof[b] = prod_{k != b} tot[k] and hands the host only their total
    // (one inversion there, ~1 us, instead of Montgomery's trick over every block product: ~3
    // multiplies per block, 40 us for 512 blocks, with the GPU idle).
    // tags (round 6): each block publishes its product as eight (epoch << 32 | limb) words and
    // arrives without a fence; the last block polls the words until they carry this launch's epoch.
    // An agent-scope fence per block writes back its XCD's whole L2 first -- with 512 blocks that
    // was most of the kernel (profiles/r06/verkle/fence_free/).
    using F = BN254Fq;
    __shared__ uint32_t s_last;
    __shared__ fe<F> spre[256], ssuf[256];
    const uint32_t tid = threadIdx.x, nb = gridDim.x;
    const uint64_t tag = (uint64_t)epoch << 32;
    if (tid == 0) {
        if (tags) {
            const fe<F> mine = tot[blockIdx.x];  // (this thread's own store in norm_prep_block)
#pragma unroll
            for (int k = 0; k < F::N; k++)
                __hip_atomic_store(&tags[(size_t)F::N * blockIdx.x + k], tag | mine.v[k], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __threadfence();  // this block's product before its arrival
        }
        s_last = atomicAdd(counter, 1u) == nb - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!s_last) return;
    if (!tags) __threadfence();
    auto load = [&](uint32_t b) {  // another block's product: through the coherent path
        fe<F> v;
        if (tags) {  // every block stored its words before it arrived: the wait is short (bounded anyway)
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                bool all = true;
#pragma unroll
                for (int k = 0; k < F::N; k++) {
                    const uint64_t w = __hip_atomic_load(&tags[(size_t)F::N * b + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    v.v[k] = (uint32_t)w;
                    all = all && (w & 0xffffffff00000000ull) == tag;
                }
                if (all || __builtin_amdgcn_s_memrealtime() - t0 > 1000000ull) break;  // (10 ms)
            }
            return v;
        }
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&tot[b]);
#pragma unroll
        for (int k = 0; k < F::N; k++) v.v[k] = __hip_atomic_load(&src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return v;
    };
    const uint32_t per = (nb + 255) / 256, b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
    fe<F> seg = fe_one<F>();
    for (uint32_t b = b1; b-- > b0;) {  // suffix products inside the segment, parked in cof
        cof[b] = seg;
        seg = fe_mul<F>(load(b), seg);
    }
    spre[tid] = seg;
    ssuf[tid] = seg;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {
        fe<F> p = spre[tid], q = ssuf[tid];
        if (tid >= off) p = fe_mul<F>(spre[tid - off], p);
        if (tid + off < 256) q = fe_mul<F>(q, ssuf[tid + off]);
        __syncthreads();
        spre[tid] = p;
        ssuf[tid] = q;
        __syncthreads();
    }
    fe<F> run = tid > 0 ? spre[tid - 1] : fe_one<F>();           // the segments before this one
    const fe<F> after = tid < 255 ? ssuf[tid + 1] : fe_one<F>();  // and after it
    for (uint32_t b = b0; b < b1; b++) {
        cof[b] = fe_mul<F>(fe_mul<F>(run, cof[b]), after);
        run = fe_mul<F>(run, load(b));
    }
    if (tid == 0) {
        *total = spre[255];
        *counter = 0;  // for the next launch (stream-ordered after this one)
        __threadfence_system();
        __hip_atomic_store(&flags[0], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <class C>
__global__ void __launch_bounds__(256) k_norm_finish(const typename C::Acc* __restrict__ in, size_t count,
                                                    const fe<typename C::F>* __restrict__ others,
                                                    const fe<typename C::F>* __restrict__ binv,
                                                    typename C::Aff* __restrict__ out_aff,
                                                    uint32_t* __restrict__ out_canon, uint8_t* __restrict__ out_inf) {
    using F = typename C::F;
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= count) return;
    const typename C::Acc a = in[j];
    bool ident = C::is_zero(a);
    const fe<F> iz = fe_mul<F>(binv[blockIdx.x], others[j]);
    fe<F> x, y;
    if constexpr (C::is_te) {
        x = fe_mul<F>(a.X, iz);
        y = fe_mul<F>(a.Y, iz);
        ident = fe_is_zero<F>(x) && fe_eq<F>(y, fe_one<F>());
    } else {
        fe<F> t = fe_mul<F>(iz, a.zz);  // 1/Z
        x = fe_mul<F>(a.x, fe_sqr<F>(t));
        y = fe_mul<F>(a.y, iz);
    }
    if (out_aff) {
        typename C::Aff r;
        r.x = x;
        r.y = y;
        if constexpr (C::is_te) r.kt = fe_mul<F>(fe_mul<F>(x, y), C::d());
        out_aff[j] = r;
    }
    if (out_canon) {
        fe<F> cx = fe_from_mont<F>(x), cy = fe_from_mont<F>(y);
        if (ident && !C::is_te) {
            cx = fe_zero<F>();
            cy = fe_zero<F>();
        }
#pragma unroll
        for (int k = 0; k < F::N; k++) {
            out_canon[j * 2 * F::N + k] = cx.v[k];
            out_canon[j * 2 * F::N + F::N + k] = cy.v[k];
        }
    }
    if (out_inf) out_inf[j] = ident ? 1 : 0;
}

// A finish kernel queued before the host has its inverse(s) (normalize_rows_items): lane 0 of block
// 0 waits for `flag` == epoch in fine-grained page-locked memory and hands it on through `relay` in
// device memory, where the other blocks wait -- with the total's inverse itself in the device-scan
// form: 512 blocks reading the same page-locked words over PCIe were served one after another,
// ~0.8 us per block, 0.4 ms for the 131,072-row level (measured, profiles/r06/verkle/norm_early/).
// In the per-block form each block reads its own inverse there. Every wait is bounded on the
// 100 MHz clock: past `limit` ticks block 0 (or a block that never saw the relay) inverts the
// value itself (prod: the block products or their total, written by the prep kernel), so the
// kernel ends whatever the host does -- it only gets slower.
struct NormGo {
    const uint32_t* flag = nullptr;  // null: the inverses were written before the launch
    uint64_t* relay = nullptr;       // 9 device words block 0 hands the go on through
    uint32_t epoch = 0;
    uint32_t per_block = 0;             // 1: inv[b] = 1 / prod[b] per block; 0: inv[0] = 1 / prod[0] (the total)
    const fe<BN254Fq>* prod = nullptr;  // what the host inverts (device view of the page-locked staging)
    const fe<BN254Fq>* inv = nullptr;   // where the host writes the inverse(s)
    uint64_t limit = 0;
    uint64_t* dbg = nullptr;  // VKZG_NORM_DEBUG: per block (start, seen or timed out, seen) on the 100 MHz clock
};
// (four 64-bit loads: page-locked host memory is read over PCIe uncached)
__device__ __forceinline__ fe<BN254Fq> load_fe_sys(const fe<BN254Fq>* p) {
    static_assert(BN254Fq::N == 8, "");
    fe<BN254Fq> v;
    uint64_t* src = const_cast<uint64_t*>(reinterpret_cast<const uint64_t*>(p));
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t w = __hip_atomic_load(&src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        v.v[2 * k] = (uint32_t)w;
        v.v[2 * k + 1] = (uint32_t)(w >> 32);
    }
    return v;
}

// verkle rows (BN254): canonical affine point, identity flag and to_data_item of row j stored at
// dst[j] (dst null: at j) -- straight into the tree's device mirror
__global__ void __launch_bounds__(256) k_norm_finish_vk(const BN254G1::Acc* __restrict__ rows, size_t count,
                                                       const fe<BN254Fq>* __restrict__ others,
                                                       const fe<BN254Fq>* __restrict__ binv,
                                                       const uint32_t* __restrict__ dst, uint64_t* __restrict__ out_xy,
                                                       uint8_t* __restrict__ out_inf, uint64_t* __restrict__ out_item,
                                                       const fe<BN254Fq>* __restrict__ tinv, NormGo go) {
    using F = BN254Fq;
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    __shared__ fe<F> s_bi;
    if (go.flag) {  // (uniform: every thread of the block reaches the barrier)
        if (threadIdx.x == 0) {
            const uint32_t k = go.per_block ? blockIdx.x : 0u;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            // relay words in device memory, each (epoch << 32) | payload, so a reader needs no ordering
            // between them and the writer no release (an agent-scope release writes back the whole
            // L2 of block 0's XCD first): [0, 8) the total's inverse, [8] whether the host answered
            uint64_t* rl = go.relay;
            const uint64_t tag = (uint64_t)go.epoch << 32;
            bool host = false, have = false, seen = false;
            fe<F> v;
            if (blockIdx.x == 0) {
                uint32_t* flag = const_cast<uint32_t*>(go.flag);
                for (;;) {
                    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == go.epoch) {
                        host = true;
                        break;
                    }
                    if (__builtin_amdgcn_s_memrealtime() - t0 > go.limit) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                seen = true;
                if (!go.per_block) {  // the one inverse: read over PCIe once, handed on in device memory
                    v = host ? load_fe_sys(go.inv) : fe_inv_bin<F>(load_fe_sys(go.prod));
                    have = true;
#pragma unroll
                    for (int i = 0; i < F::N; i++)
                        __hip_atomic_store(&rl[i], tag | v.v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    __hip_atomic_store(&rl[8], tag | (host ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                const int nw = go.per_block ? 1 : F::N;
                uint64_t* src = go.per_block ? rl + 8 : rl;
                uint64_t w[F::N];
                for (;;) {
                    bool all = true;
                    for (int i = 0; i < nw; i++) {
                        w[i] = __hip_atomic_load(&src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        all = all && (w[i] >> 32) == go.epoch;
                    }
                    if (all) {
                        seen = true;
                        break;
                    }
                    if (__builtin_amdgcn_s_memrealtime() - t0 > go.limit) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                if (seen && go.per_block) host = (w[0] & 1u) != 0;
                if (seen && !go.per_block) {
#pragma unroll
                    for (int i = 0; i < F::N; i++) v.v[i] = (uint32_t)w[i];
                    have = true;
                }
            }
            if (go.dbg) {
                go.dbg[3 * blockIdx.x] = t0;
                go.dbg[3 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
                go.dbg[3 * blockIdx.x + 2] = (seen ? 1u : 0u) | (host ? 2u : 0u);
            }
            // per block: its own inverse from the host (distinct addresses), or made here
            if (!have) v = host ? load_fe_sys(go.inv + k) : fe_inv_bin<F>(load_fe_sys(go.prod + k));
            s_bi = go.per_block ? v : fe_mul<F>(v, binv[blockIdx.x]);
        }
        __syncthreads();
    }
    if (j >= count) return;
    const BN254G1::Acc a = rows[j];
    const bool ident = BN254G1::is_zero(a);
    // the block's inverse: binv[b], or (device scan) the cofactor times the total's inverse, or
    // (queued early) what lane 0 got above
    const fe<F> bi = go.flag ? s_bi : tinv ? fe_mul<F>(*tinv, binv[blockIdx.x]) : binv[blockIdx.x];
    const fe<F> iz = fe_mul<F>(bi, others[j]);
    const fe<F> t = fe_mul<F>(iz, a.zz);  // 1/Z
    fe<F> cx = fe_from_mont<F>(fe_mul<F>(a.x, fe_sqr<F>(t))), cy = fe_from_mont<F>(fe_mul<F>(a.y, iz));
    if (ident) cx = cy = fe_zero<F>();
    const size_t o = dst ? dst[j] : j;
    memcpy(out_xy + 8 * o, cx.v, 32);
    memcpy(out_xy + 8 * o + 4, cy.v, 32);
    out_inf[o] = ident ? 1 : 0;
    const fe<BN254Fr> it = to_data_item_canon(cx, cy, ident);
    memcpy(out_item + 4 * o, it.v, 32);
}

// d_in (count accumulators) -> affine / canonical outputs; synchronises the stream once
template <class C>
static int normalize_split(vc_ctx* ctx, const typename C::Acc* d_in, size_t count, typename C::Aff* out_aff,
                           uint32_t* out_canon, uint8_t* out_inf) {
    using F = typename C::F;
    if (count == 0) return VC_OK;
    const size_t nblk = (count + 255) / 256;
    DevBuf others(ctx), tot(ctx);
    VK_TRY(others.ensure(count * sizeof(fe<F>)));
    VK_TRY(tot.ensure(nblk * sizeof(fe<F>)));
    VK_TRY(ctx->pin_norm.ensure(2 * nblk * sizeof(fe<F>)));
    fe<F>* h = ctx->pin_norm.as<fe<F>>();
    VK_LAUNCH(ctx, "norm_prep", (k_norm_prep<C>), nblk, 256, 0, d_in, count, others.as<fe<F>>(), tot.as<fe<F>>());
    VK_CHECK_HIP(hipMemcpyAsync(h, tot.p, nblk * sizeof(fe<F>), hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    // Montgomery's trick over the block products (never zero: identities count as 1)
    fe<F>* inv = h + nblk;
    inv[0] = h[0];
    for (size_t b = 1; b < nblk; b++) inv[b] = fe_mul<F>(inv[b - 1], h[b]);
    fe<F> run = fe_inv_bin<F>(inv[nblk - 1]);
    for (size_t b = nblk - 1; b > 0; b--) {
        const fe<F> ib = fe_mul<F>(run, inv[b - 1]);
        run = fe_mul<F>(run, h[b]);
        inv[b] = ib;
    }
    inv[0] = run;
    VK_CHECK_HIP(hipMemcpyAsync(tot.p, inv, nblk * sizeof(fe<F>), hipMemcpyHostToDevice, ctx->stream));
    VK_LAUNCH(ctx, "norm_finish", (k_norm_finish<C>), nblk, 256, 0, d_in, count, others.as<fe<F>>(),
              tot.as<fe<F>>(), out_aff, out_canon, out_inf);
    // the pinned staging is reused by the next call: the copy above must have left it
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}

// ------------------------------------------------------------------ the batched commit
// Chunk-major runs: the width is cut into nch chunks of <= K bases and run r = chunk * batch + g
// adds commit g's items of chunk `chunk`. The 64 lanes of a wave are 64 commits at the same base
// and window, so each gather instruction stays inside one (base, window) block of the table
// (3 MB at c = 16) instead of touching 64 blocks spread over the whole table (GBs): far fewer
// distinct pages per instruction, and the identity-base skip is wave-uniform.
template <class C, class Fr>
__global__ void __launch_bounds__(256) VK_COMMIT_OCC k_fb_commit_cm(const FbE<C>* __restrict__ tab,
                                                     const uint8_t* __restrict__ inf, uint32_t width,
                                                     FbGeom fg, const uint32_t* __restrict__ sc,
                                                     uint32_t batch, int mont, uint32_t K, uint32_t nruns,
                                                     typename Fast29<C>::type::Acc* __restrict__ piece) {
    using FC = typename Fast29<C>::type;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nruns) return;
    const uint32_t chunk = r / batch, g = r - chunk * batch;
    const int W = fg.W;
    const uint32_t i0 = chunk * K, i1 = min(i0 + K, width);
    typename FC::Acc acc = FC::zero();
    for (uint32_t i = i0; i < i1; i++) {
        if (inf[i]) continue;
        FbDigits<Fr> dg;
        dg.s = load_scalar_fb<Fr>(sc, (size_t)g * width + i);
        if (mont) dg.s = fe_from_mont<Fr>(dg.s);
        const FbE<C>* ti = tab + (size_t)i * fg.stride();
        int32_t dn = dg.next(fg.width(0));
        typename FC::Aff Pn = ti[dn != 0 ? (uint32_t)(dn < 0 ? -dn : dn) - 1 : 0].u;
        for (int w = 0; w < W; w++) {
            const int32_t d = dn;
            const typename FC::Aff P = Pn;
            if (w + 1 < W) {
                dn = dg.next(fg.width(w + 1));
                Pn = ti[fg.off(w + 1) + (dn != 0 ? (uint32_t)(dn < 0 ? -dn : dn) - 1 : 0)].u;
            }
            if (d != 0) acc = FC::madd(acc, P, d < 0);
        }
    }
    piece[r] = acc;
}

// commit g = sum over chunks of the raw pieces piece[chunk * batch + g]: a thread per commit
// (coalesced across g) for large batches, or a wave per commit (lanes fold a strided share,
// then an xor butterfly) for small ones, which the chip spreads over up to `width` chunks per
// commit: a serial chain of 257 adds cost ~2 ms (IPA prover rounds)
template <class C>
__global__ void __launch_bounds__(256) k_fb_combine_cm(const typename Fast29<C>::type::Acc* __restrict__ piece,
                                                      uint32_t nch, uint32_t batch, typename C::Acc* __restrict__ out) {
    using FC = typename Fast29<C>::type;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= batch) return;
    typename FC::Acc acc = piece[g];
    for (uint32_t k = 1; k < nch; k++) acc = FC::add(acc, piece[(size_t)k * batch + g]);
    out[g] = FC::store(acc);
}
// G = 2^lgG lanes per commit (consecutive lanes of one wave): each folds a strided share of the
// nch pieces, then lgG xor levels -- ceil(nch / G) + lgG serial adds. G grows while the lanes
// still fit one wave per SIMD: 10k width-256 commits (13 chunks) take 4 lanes each, 5 adds
// instead of the 12 of a thread per commit on 157 waves
template <class C>
__global__ void __launch_bounds__(256) k_fb_combine_grp(const typename Fast29<C>::type::Acc* __restrict__ piece,
                                                       uint32_t nch, uint32_t batch, uint32_t lgG,
                                                       typename C::Acc* __restrict__ out) {
    using FC = typename Fast29<C>::type;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, g = gid >> lgG, j = gid & ((1u << lgG) - 1);
    const uint32_t G = 1u << lgG, nk = (nch + G - 1) / G;
    typename FC::Acc v = FC::zero();
    for (uint32_t it = 0; it < nk + lgG; it++) {  // one add call site; every lane runs the shuffles
        typename FC::Acc o;
        if (it < nk) {
            const uint32_t k = j + it * G;
            o = (g < batch && k < nch) ? piece[(size_t)k * batch + g] : FC::zero();
        } else {
            o = shfl_xor_pod(v, 1u << (it - nk));
        }
        v = FC::add(v, o);
    }
    if (g < batch && j == 0) out[g] = FC::store(v);
}
template <class C>
__global__ void __launch_bounds__(64) k_fb_combine_wave(const typename Fast29<C>::type::Acc* __restrict__ piece,
                                                       uint32_t nch, uint32_t batch, typename C::Acc* __restrict__ out) {
    using FC = typename Fast29<C>::type;
    const uint32_t g = blockIdx.x, lane = threadIdx.x;
    uint32_t span = 1, lg = 0;
    while (span < nch && span < 64) {
        span <<= 1;
        lg++;
    }
    const uint32_t nk = (nch + 63) / 64;
    typename FC::Acc v = FC::zero();
    for (uint32_t it = 0; it < nk + lg; it++) {  // one add call site
        typename FC::Acc o;
        if (it < nk) {
            const uint32_t k = lane + it * 64;
            o = k < nch ? piece[(size_t)k * batch + g] : FC::zero();
        } else {
            o = shfl_xor_pod(v, 1u << (it - nk));
        }
        v = FC::add(v, o);
    }
    if (lane == 0) out[g] = FC::store(v);
}
// ---- latency path for small batches (the IPA prover's L/R, multiproof D/E): every thread
// adds the table points of WPT windows of one base, then a wave butterfly and an LDS step
// fold the block to one partial; k_fb_combine_small adds a commit's few block partials.
// Serial depth WPT + 8 + blocks-per-commit adds instead of W + width (persistent path at K = 1).
// windows per thread of the latency path. 1 is best by far (IPA prover L/R, width 257, c = 8:
// 111 us per launch vs 469 / 658 us at 2 / 4): a lone wave executing a mixed add's ~25 KB of
// straight-line code once runs on cold instruction-cache misses, so any serial madd beyond the
// first costs ~0.35 ms; one (base, window) point per thread leaves only the looped butterfly.
constexpr int FB_WPT = 1;
static int fb_wpt() { return FB_WPT; }

template <class C, class Fr>
__global__ void __launch_bounds__(256) k_fb_commit_small(const FbE<C>* __restrict__ tab,
                                                        const uint8_t* __restrict__ inf, uint32_t width, FbGeom fg,
                                                        const uint32_t* __restrict__ sc, int mont,
                                                        uint32_t bpc, int wpt, StrideCols cols, IpaRows ipa,
                                                        typename C::Acc* __restrict__ part,
                                                        uint32_t* __restrict__ flags, uint32_t epoch) {
    using FC = typename Fast29<C>::type;
    const uint32_t g = blockIdx.x / bpc, blk = blockIdx.x % bpc;
    const int W = fg.W;
    const uint32_t WG = (uint32_t)(W + wpt - 1) / wpt;
    const uint32_t j = blk * 256 + threadIdx.x;
    const uint32_t i = j / WG, wg = j % WG;
    typename FC::Acc fa = FC::zero();
    // compacted rows (cols.half != 0): commit g's item i is a table base of a strided pattern
    // (computed: a list in host memory cost a dependent PCIe read per thread, +7 us per launch)
    const uint32_t base = cols.half ? cols.base(g, i) : i;
    // the IPA rows (IpaRows): this round's coefficient of item i, folded and stored by L's window-0
    // thread for the next round -- identity bases included -- then the item's scalar
    fe<Fr> ipa_s = fe_zero<Fr>();
    if (ipa.a != nullptr && i < width) {
        const uint32_t p = g >> 1;
        if (i < ipa.N) {
            fe<Fr> c = load_scalar_fb<Fr>(ipa.coeff_in, (size_t)p * ipa.N + i);
            if (ipa.fold && (i % ipa.m_prev) < ipa.h_prev) c = fe_mul<Fr>(c, load_scalar_fb<Fr>(ipa.x, p));
            if ((g & 1) == 0 && wg == 0) {
                uint4* o = reinterpret_cast<uint4*>(ipa.coeff_out + 8 * ((size_t)p * ipa.N + i));
                o[0] = make_uint4(c.v[0], c.v[1], c.v[2], c.v[3]);
                o[1] = make_uint4(c.v[4], c.v[5], c.v[6], c.v[7]);
            }
            const uint32_t jj = i % ipa.m;
            const bool on = (g & 1) ? jj < ipa.h : jj >= ipa.h;
            if (on)
                ipa_s = fe_mul<Fr>(load_scalar_fb<Fr>(ipa.a, (size_t)p * ipa.N + ((g & 1) ? jj + ipa.h : jj - ipa.h)), c);
        } else {
            ipa_s = load_scalar_fb<Fr>(ipa.q, g);
        }
    }
    if (i < width && !inf[base]) {
        FbDigits<Fr> dg;
        dg.s = ipa.a != nullptr ? ipa_s : load_scalar_fb<Fr>(sc, (size_t)g * width + i);
        if (mont) dg.s = fe_from_mont<Fr>(dg.s);
        const FbE<C>* ti = tab + (size_t)base * fg.stride();
        const int wb = (int)wg * wpt, we = min(W, wb + wpt);
        for (int w = 0; w < we; w++) {
            const int32_t d = dg.next(fg.width(w));
            if (w >= wb && d != 0) fa = FC::madd(fa, ti[fg.off(w) + (uint32_t)(d < 0 ? -d : d) - 1].u, d < 0);
        }
    }
    fb_block_sum_store<C>(fa, &part[blockIdx.x]);
    // zero-copy completion: the block's partial (written by thread 0 above) is made visible system
    // wide, then its flag takes this launch's epoch -- the host polls the flags instead of waiting
    // for the stream (fb_commit_t)
    if (flags != nullptr && threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(&flags[blockIdx.x], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <class C>
__global__ void k_fb_combine_small(const typename C::Acc* __restrict__ part, uint32_t bpc, uint32_t batch,
                                   typename C::Acc* __restrict__ out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= batch) return;
    typename C::Acc acc = part[(size_t)g * bpc];
    for (uint32_t b = 1; b < bpc; b++) acc = C::add(acc, part[(size_t)g * bpc + b]);
    out[g] = acc;
}

// lanes resident in one round for a kernel (occupancy x CUs x block)
template <class Kern>
static uint32_t resident_lanes(Kern k, int block) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, block, 0) != hipSuccess) return 0;
    return (uint32_t)(cus * per_cu * block);
}

// ------------------------------------------------------------------ host drivers
// scalar bits of the curve's group order (signed digits need windows covering bits + 1)
template <class C>
using FrOf = typename std::conditional<std::is_same<C, BN254G1>::value, BN254Fr,
                                       typename std::conditional<std::is_same<C, BLS381G1>::value, BLS381Fr,
                                                                 BandFr>::type>::type;

// windows = 0: uniform c-bit windows; otherwise `windows` windows of c or c + 1 bits (the last
// bits + 1 - c windows wide), which must cover the scalar's bits + 1
template <class C>
static int fb_precompute_t(vc_ctx* ctx, Table* t, int c, int windows) {
    using Acc = typename C::Acc;
    using Aff = typename C::Aff;
    using Fr = FrOf<C>;
    if (c < 4 || c > 20 || windows < 0) return VC_E_INVALID;
    const uint32_t n = (uint32_t)t->n;
    int W = (Fr::BITS + 1 + c - 1) / c, big = 0;
    if (windows > 0 && windows < W) {
        big = Fr::BITS + 1 - c * windows;
        if (big > windows || c == 20) return VC_E_INVALID;  // needs wider windows than c + 1
        W = windows;
    }
    const FbGeom g{c, W, big};
    const uint32_t NBk = 1u << (c - 1), NBmax = big ? 2 * NBk : NBk;
    if (t->fb_c == c && t->fb_W == W && t->fb_big == big && t->fb.p) return VC_OK;
    t->fb.release();
    t->fb_c = 0;
    t->fb_auto = false;  // (fb_commit_t marks its own first-use builds)
    VK_TRY(t->fb.ensure(std::max<size_t>((size_t)n * g.stride(), 1) * sizeof(FbE<C>)));
    DevBuf Q, tmp, aff_w;
    VK_TRY(Q.ensure(std::max<uint32_t>(n, 1) * sizeof(Acc)));
    VK_TRY(tmp.ensure(std::max<size_t>((size_t)n * NBmax, 1) * sizeof(Acc)));
    VK_TRY(aff_w.ensure(std::max<size_t>((size_t)n * NBmax, 1) * sizeof(Aff)));
    for (int w = 0; w < W; w++) {
        const uint32_t NBw = 1u << (g.width(w) - 1);
        const uint32_t CH = NBw >= 64 ? 64 : NBw;
        const uint32_t nch = (NBw + CH - 1) / CH;
        // Q = 2^(bits below window w) G: the previous window's width more doublings
        VK_LAUNCH(ctx, "fb_shift", (k_fb_shift<C>), (n + 255) / 256, 256, 0, Q.as<Acc>(),
                  t->bases.as<Aff>(), n, w == 0 ? 0 : g.width(w - 1), w == 0 ? 1 : 0);
        VK_LAUNCH(ctx, "fb_fill", (k_fb_fill<C>), ((size_t)n * nch + 127) / 128, 128, 0, Q.as<Acc>(), n,
                  NBw, CH, tmp.as<Acc>());
        size_t cnt = (size_t)n * NBw;
        VK_LAUNCH(ctx, "fb_normalize", (k_normalize<C>), (cnt + 255) / 256, 256, 0, tmp.as<Acc>(), cnt,
                  aff_w.as<Aff>(), (uint32_t*)nullptr, (uint8_t*)nullptr);
        VK_LAUNCH(ctx, "fb_place", (k_fb_place<C>), (cnt + 255) / 256, 256, 0, aff_w.as<Aff>(), n, NBw, g, w,
                  t->fb.as<FbE<C>>());
    }
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    t->fb_c = c;
    t->fb_W = W;
    t->fb_big = big;
    return VC_OK;
}

// window bits of the fixed-base tables a commit builds on first use (a table without
// vc_fixed_base_precompute: the IPA CRS of the prover / verifier, the multiproof's D / E): the
// widest c <= 16 whose table fits what is left of the context's budget for such tables
// (VKZG_FB_BUDGET_GB, default 20 GB of the card's 288, less the ones built before and still held)
// and into the device's free memory less a 4 GB margin (hipMemGetInfo), at least 8; a build that
// still fails for memory retries one window bit narrower, down to 8 (fb_commit_t).
// Fewer windows mean fewer table points per commit, hence fewer latency-path blocks and block
// partials: the 257-point IPA CRS at c = 16 (16 windows, 17.2 GB) proves in 0.64 ms against 0.73 at
// c = 8 (32 windows, 134 MB), the multiproof finish 0.99 against 1.15 ms (profiles/r05/fb_default_c/).
// VKZG_FB_C_DEFAULT (read once; A/B probe) fixes c.
template <class Fr>
static double fb_auto_bytes(size_t n, int c) {
    const size_t W = (size_t)(Fr::BITS + 1 + c - 1) / c;
    return (double)n * (double)W * (double)(1u << (c - 1)) * 128.0;
}
template <class Fr>
static int fb_default_c(size_t n, size_t used) {
    static const int forced = getenv("VKZG_FB_C_DEFAULT") ? atoi(getenv("VKZG_FB_C_DEFAULT")) : 0;
    static const double budget_gb = getenv("VKZG_FB_BUDGET_GB") ? atof(getenv("VKZG_FB_BUDGET_GB")) : 20.0;
    if (forced >= 4 && forced <= 20) return forced;
    double limit = budget_gb * 1e9 - (double)used;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) limit = std::min(limit, (double)free_b - 4e9);
    for (int c = 16; c > 8; c--)
        if (fb_auto_bytes<Fr>(n, c) <= limit) return c;
    return 8;
}

template <class C, class Fr>
static int fb_commit_t(vc_ctx* ctx, Table* t, size_t width, const void* d_sc, size_t batch, int mont,
                       void* d_out_xy, uint8_t* d_out_inf, uint64_t* h_out_xy, uint8_t* h_out_inf, bool* on_host,
                       const PinBuf* pin_sc, const std::function<void()>* overlap, const StrideCols* cols,
                       const IpaRows* ipa) {
    using Acc = typename C::Acc;
    const bool with_cols = cols && cols->half;
    if (width > t->n && !with_cols) return VC_E_RANGE;
    if (with_cols && (size_t)cols->extra >= t->n) return VC_E_RANGE;
    if (with_cols && cols->base(0, cols->n_main - 1) >= t->n) return VC_E_RANGE;
    if (t->fb_c == 0) {
        int c = fb_default_c<Fr>(t->n, ctx->fb_auto_used());
        int st = fb_precompute_t<C>(ctx, t, c, 0);
        while (st == VC_E_OOM && c > 8) {  // another context or caller took the memory: narrower
            (void)hipGetLastError();
            st = fb_precompute_t<C>(ctx, t, --c, 0);
        }
        VK_TRY(st);
        t->fb_auto = true;
    }
    if (batch == 0) {
        if (overlap && *overlap) (*overlap)();
        return VC_OK;
    }
    VK_TRY(ctx->ws[WS_OUT].ensure(batch * sizeof(Acc)));
    // resident lanes of this context's device (cached per ctx: the Guard's mutex serialises it)
    if (!ctx->fb_lanes) ctx->fb_lanes = resident_lanes(k_fb_commit_cm<C, Fr>, 256);
    const size_t items = batch * width;
    const size_t lanes = ctx->fb_lanes ? ctx->fb_lanes : 131072;
    const FbGeom fg = t->fb_geom();
    const int W = fg.W;
    const int wpt = fb_wpt();
    const size_t WG = (size_t)(W + wpt - 1) / wpt;
    const bool small = items * WG <= lanes && batch <= 64;
    if ((with_cols || ipa) && !small) return VC_E_INVALID;  // compacted / IPA rows: the latency path only
    if (ipa && (with_cols || width != (size_t)ipa->N + 1 || batch % 2)) return VC_E_INVALID;
    // zero-copy on the latency path (VKZG_ZERO_COPY, A/B probe: bit 0 partials, bit 1 scalars):
    // the kernel reads host-pinned scalars and writes its block partials to fine-grained host
    // memory over PCIe instead of a copy engine moving them before / after it
    static const int zc = getenv("VKZG_ZERO_COPY") ? atoi(getenv("VKZG_ZERO_COPY")) : 3;
    if (pin_sc) {
        if (small && (zc & 2)) {
            d_sc = pin_sc->dp;
        } else {
            VK_TRY(ctx->ws[WS_SCALARS].ensure(items * 32));
            VK_CHECK_HIP(hipMemcpyAsync(ctx->ws[WS_SCALARS].p, pin_sc->p, items * 32, hipMemcpyHostToDevice,
                                        ctx->stream));
            d_sc = ctx->ws[WS_SCALARS].p;
        }
    }
    if (small) {  // small batch: latency path
        const uint32_t bpc = (uint32_t)((width * WG + 255) / 256);
        // VKZG_HOST_TIMING=1: launch-to-readback, host adds and normalisation on stderr (probe)
        static const bool timing = getenv("VKZG_HOST_TIMING") && atoi(getenv("VKZG_HOST_TIMING")) != 0;
        auto now_us = [] {
            return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
        };
        const double t0 = timing ? now_us() : 0.0;
        const size_t part_bytes = (size_t)batch * bpc * sizeof(Acc);
        const uint32_t nblk = (uint32_t)(batch * bpc);
        // zero-copy partials: the blocks' completion flags follow them in the fine-grained buffer
        // (VKZG_SMALL_POLL=0, read once: wait for the stream instead)
        static const bool poll_env = !(getenv("VKZG_SMALL_POLL") && atoi(getenv("VKZG_SMALL_POLL")) == 0);
        const bool poll = poll_env && (zc & 1);
        const size_t flag_off = (part_bytes + 63) / 64 * 64;
        VK_TRY(ctx->pin_small.ensure(flag_off + (size_t)nblk * 4));
        if (!(zc & 1)) VK_TRY(ctx->ws[WS_PIECE].ensure(part_bytes));
        Acc* d_part = (zc & 1) ? static_cast<Acc*>(ctx->pin_small.dp) : ctx->ws[WS_PIECE].as<Acc>();
        volatile uint32_t* hflags = reinterpret_cast<volatile uint32_t*>(static_cast<uint8_t*>(ctx->pin_small.p) + flag_off);
        uint32_t* dflags = poll ? reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pin_small.dp) + flag_off) : nullptr;
        const uint32_t epoch = ++ctx->small_epoch == 0 ? ++ctx->small_epoch : ctx->small_epoch;  // never 0
        if (poll)  // (fresh page-locked memory holds anything: no stale flag may match)
            for (uint32_t b = 0; b < nblk; b++) hflags[b] = 0;
        VK_LAUNCH(ctx, "fb_commit_small", (k_fb_commit_small<C, Fr>), batch * bpc, 256, 0, t->fb.as<FbE<C>>(),
                  t->inf.as<uint8_t>(), (uint32_t)width, fg, reinterpret_cast<const uint32_t*>(d_sc), mont,
                  bpc, wpt, with_cols ? *cols : StrideCols{}, ipa ? *ipa : IpaRows{}, d_part, dflags, epoch);
        // the few block partials are added and normalised on the host: a lone GPU lane pays
        // ~10 us per serial EC add and ~160 us per field inversion, the host ~1 us / ~20 us
        // (pinned read-back; a caller that wants host results -- h_out_xy -- gets them without the
        // upload / second read-back round trip)
        const Acc* parts = ctx->pin_small.as<Acc>();
        if (!(zc & 1))
            VK_CHECK_HIP(hipMemcpyAsync(ctx->pin_small.p, ctx->ws[WS_PIECE].p, part_bytes, hipMemcpyDeviceToHost,
                                        ctx->stream));
        if (overlap && *overlap) (*overlap)();
        bool seen = false;
        // the partials serially on this thread (the host pool's wake-up cost more than the ~23 us
        // of adds of the IPA prover's 2 x 33 partials: prove 0.89 -> 1.07 ms); while polling, each
        // block's partial is added as soon as its flag arrives, so the adds overlap the blocks
        // that finish later. Then one batched inversion.
        std::vector<Acc> sums(batch);
        // VKZG_SMALL_INCR=0 (read once; A/B probe): add the partials after the last flag instead
        static const bool incr = !(getenv("VKZG_SMALL_INCR") && atoi(getenv("VKZG_SMALL_INCR")) == 0);
        if (poll) {  // every block's flag at this epoch: the partials are in host memory
            std::vector<uint8_t> done(nblk, 0), have(batch, 0);
            uint32_t ndone = 0;
            const auto w0 = std::chrono::steady_clock::now();
            for (uint32_t spins = 0;; spins++) {
                for (uint32_t b = 0; b < nblk; b++) {
                    if (done[b] || hflags[b] != epoch) continue;
                    if (incr) {
                        std::atomic_thread_fence(std::memory_order_acquire);
                        const uint32_t g = b / bpc;
                        sums[g] = have[g] ? C::add(sums[g], parts[b]) : parts[b];
                        have[g] = 1;
                    }
                    done[b] = 1;
                    ndone++;
                }
                if (ndone == nblk) {
                    seen = true;
                    break;
                }
                // bounded: past 20 ms (a first launch loading its code, or a fault) wait for the
                // stream, which also reports any error
                if ((spins & 1023) == 1023 &&
                    std::chrono::steady_clock::now() - w0 > std::chrono::milliseconds(20))
                    break;
                _mm_pause();
            }
        }
        const double t1 = timing ? now_us() : 0.0;
        if (!seen) VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        if (!seen || !incr) {
            std::atomic_thread_fence(std::memory_order_acquire);
            for (size_t g = 0; g < batch; g++) {
                Acc a = parts[g * bpc];
                for (uint32_t b = 1; b < bpc; b++) a = C::add(a, parts[g * bpc + b]);
                sums[g] = a;
            }
        }
        const int nl = (int)(C::F::N / 2);
        std::vector<uint64_t> oxy(h_out_xy ? 0 : (size_t)batch * 2 * nl);
        std::vector<uint8_t> oinf(h_out_xy ? 0 : batch);
        uint64_t* rxy = h_out_xy ? h_out_xy : oxy.data();
        uint8_t* rinf = h_out_xy ? h_out_inf : oinf.data();
        const double t2 = timing ? now_us() : 0.0;
        VK_TRY(acc_to_affine_batch(ctx->curve, reinterpret_cast<const uint32_t*>(sums.data()), batch, rxy, rinf));
        if (timing)
            fprintf(stderr, "[fb_small] %zu x %u partials: launch..last flag (adds overlapped) %.1f us, rest %.1f us, affine %.1f us\n",
                    batch, bpc, t1 - t0, t2 - t1, now_us() - t2);
        if (h_out_xy) {
            *on_host = true;
            return VC_OK;
        }
        VK_CHECK_HIP(hipMemcpyAsync(d_out_xy, oxy.data(), oxy.size() * 8, hipMemcpyHostToDevice, ctx->stream));
        VK_CHECK_HIP(hipMemcpyAsync(d_out_inf, oinf.data(), batch, hipMemcpyHostToDevice, ctx->stream));
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));  // host staging vectors die on return
        return VC_OK;
    }
    // chunk-major: the chunk count minimising rounds-of-resident-lanes x items-per-run
    // (fewest chunks on ties: fewer pieces to combine)
    size_t K = width, best = SIZE_MAX;
    for (size_t nc = 1; nc <= width; nc++) {
        const size_t k = (width + nc - 1) / nc;
        if ((width + k - 1) / k != nc) continue;  // same K as a smaller chunk count
        const size_t cost = ((nc * batch + lanes - 1) / lanes) * k;
        if (cost < best) best = cost, K = k;
    }
    const size_t nch = (width + K - 1) / K;
    const size_t nruns = nch * batch;
    if (nruns >= (1ull << 31)) return VC_E_RANGE;
    VK_TRY(ctx->ws[WS_PIECE].ensure(nruns * sizeof(typename Fast29<C>::type::Acc)));
    VK_LAUNCH(ctx, "fb_commit", (k_fb_commit_cm<C, Fr>), (nruns + 255) / 256, 256, 0,
              t->fb.as<FbE<C>>(), t->inf.as<uint8_t>(), (uint32_t)width, fg,
              reinterpret_cast<const uint32_t*>(d_sc), (uint32_t)batch, mont, (uint32_t)K, (uint32_t)nruns,
              ctx->ws[WS_PIECE].as<typename Fast29<C>::type::Acc>());
    // serial adds per SIMD: a thread per commit (nch adds, batch / 64 waves) vs a wave per commit
    // (ceil(nch / 64) + log2 adds, batch waves) -- 1024 SIMDs
    size_t lg = 0;
    while ((1ull << lg) < std::min<size_t>(nch, 64)) lg++;
    const size_t cost_thread = nch * ((batch + 65535) / 65536);
    const size_t cost_wave = ((batch + 1023) / 1024) * ((nch + 63) / 64 + lg);
    // lanes per commit: grow while there are pieces to split and the lanes fit a wave per SIMD
    uint32_t lgG = 0;
    while (lgG < 6 && (2ull << lgG) <= nch && batch * (2ull << lgG) <= 65536) lgG++;
    static const int grp_env = getenv("VKZG_COMBINE_GROUP") ? atoi(getenv("VKZG_COMBINE_GROUP")) : 1;  // A/B probe
    if (grp_env && lgG > 0 && lgG < 6)
        VK_LAUNCH(ctx, "fb_combine", (k_fb_combine_grp<C>), (uint32_t)(((batch << lgG) + 255) / 256), 256, 0,
                  ctx->ws[WS_PIECE].as<typename Fast29<C>::type::Acc>(), (uint32_t)nch, (uint32_t)batch, lgG,
                  ctx->ws[WS_OUT].as<Acc>());
    else if (cost_thread <= cost_wave)
        VK_LAUNCH(ctx, "fb_combine", (k_fb_combine_cm<C>), (batch + 255) / 256, 256, 0,
                  ctx->ws[WS_PIECE].as<typename Fast29<C>::type::Acc>(), (uint32_t)nch, (uint32_t)batch,
                  ctx->ws[WS_OUT].as<Acc>());
    else
        VK_LAUNCH(ctx, "fb_combine", (k_fb_combine_wave<C>), batch, 64, 0,
                  ctx->ws[WS_PIECE].as<typename Fast29<C>::type::Acc>(), (uint32_t)nch, (uint32_t)batch,
                  ctx->ws[WS_OUT].as<Acc>());
    if (overlap && *overlap) (*overlap)();
    return normalize_split<C>(ctx, ctx->ws[WS_OUT].as<Acc>(), batch, (typename C::Aff*)nullptr,
                              reinterpret_cast<uint32_t*>(d_out_xy), d_out_inf);
}

// table <- normalised projective accumulators (device), e.g. a freshly computed SRS
template <class C>
static int table_from_acc_t(vc_ctx* ctx, Table* t, const void* d_acc, size_t n) {
    t->curve = ctx->curve;
    t->n = n;
    t->fb_c = t->fb_W = t->fb_big = 0;
    t->fb_auto = false;
    t->fb.release();
    delete t->lead;
    t->lead = nullptr;
    t->lead_k = t->lead_c = 0;
    t->fast_ok = t->phi_ok = t->win_ok = 0;
    VK_TRY(t->bases.ensure(std::max<size_t>(n, 1) * sizeof(typename C::Aff)));
    VK_TRY(t->inf.ensure(std::max<size_t>(n, 1)));
    if (n == 0) return VC_OK;
    VK_LAUNCH(ctx, "normalize_table", (k_normalize<C>), (n + 255) / 256, 256, 0,
              reinterpret_cast<const typename C::Acc*>(d_acc), n, t->bases.as<typename C::Aff>(),
              (uint32_t*)nullptr, t->inf.as<uint8_t>());
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}
int table_from_acc(vc_ctx* ctx, Table* t, const void* d_acc, size_t n) {
    switch (ctx->curve) {
        case VC_CURVE_BN254: return table_from_acc_t<BN254G1>(ctx, t, d_acc, n);
        case VC_CURVE_BLS12_381: return table_from_acc_t<BLS381G1>(ctx, t, d_acc, n);
        case VC_CURVE_BANDERSNATCH: return table_from_acc_t<Bandersnatch>(ctx, t, d_acc, n);
    }
    return VC_E_INVALID;
}

// verkle rows (BN254, device): optional old-commitment adds, then canonical affine points,
// identity flags and to_data_item values at dst[j] (k_norm_prep_vk / k_norm_finish_vk). One
// pinned round trip (the block products' inversion on the host) and no trailing synchronisation:
// the finish kernel and its H2D copy stay queued (the next call synchronises the stream -- after
// the D2H of its products -- before its host writes into pin_norm_vk, so the copy has left it).
int normalize_rows_items(vc_ctx* ctx, void* d_rows, size_t n, const uint32_t* add_ids, const uint64_t* add_xy,
                         const uint8_t* add_inf, const uint32_t* dst, uint64_t* out_xy, uint8_t* out_inf,
                         uint64_t* out_item, const std::function<void()>* overlap) {
    using F = BN254Fq;
    if (n == 0) return VC_OK;
    const size_t nblk = (n + 255) / 256;
    DevBuf others(ctx);
    VK_TRY(others.ensure(n * sizeof(fe<F>)));
    // fine-grained page-locked staging of its own, two halves used by alternate calls, each
    // [block products | inverses | flags]: the prep kernel writes the products and per-block flags
    // straight into it, the host polls the flags, writes the inverses there and the finish kernel
    // reads them in place -- no copies, no stream wait (a bounded spin; the stream wait is the
    // fallback). The previous call's finish may still read its inverses, so this call takes the
    // other half (the call before that finished: its successor's prep, queued after it, was seen
    // complete); the buffer grows only after a sync.
    // [block products | inverses | the prep's flags | the host's go word]
    const size_t flag_off = 2 * nblk * sizeof(fe<F>), go_off = flag_off + nblk * 4;
    const size_t half_bytes = (go_off + 4 + 255) / 256 * 256;
    if (ctx->pin_norm_vk.cap < 2 * half_bytes) {
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        VK_TRY(ctx->pin_norm_vk.ensure(2 * half_bytes));
    }
    const size_t half = ctx->pin_norm_vk.cap / 2 / 256 * 256;  // (>= half_bytes)
    ctx->norm_vk_parity ^= 1u;
    uint8_t* hbase = ctx->pin_norm_vk.as<uint8_t>() + ctx->norm_vk_parity * half;
    uint8_t* dbase = static_cast<uint8_t*>(ctx->pin_norm_vk.dp) + ctx->norm_vk_parity * half;
    fe<F>* h = reinterpret_cast<fe<F>*>(hbase);
    fe<F>* dh = reinterpret_cast<fe<F>*>(dbase);
    volatile uint32_t* hflags = reinterpret_cast<volatile uint32_t*>(hbase + flag_off);
    uint32_t* dflags = reinterpret_cast<uint32_t*>(dbase + flag_off);
    volatile uint32_t* hgo = reinterpret_cast<volatile uint32_t*>(hbase + go_off);
    const uint32_t epoch = ++ctx->small_epoch == 0 ? ++ctx->small_epoch : ctx->small_epoch;  // never 0
    // the finish kernel queued right behind the prep, before the host has the inverse (NormGo): its
    // blocks wait on the host's go word, so the host's inversion is no longer followed by a launch
    // (~10-20 us of idle GPU per level) and the host queues the next level's work while the prep
    // runs. VKZG_NORM_EARLY=0: launch the finish after the inversion (A/B); VKZG_NORM_EARLY_US: the
    // blocks' wait before they invert on their own.
    // (both read per call: a test sets a 1-us bound to run the blocks' own inversions)
    const char* ee = getenv("VKZG_NORM_EARLY");
    const char* eu = getenv("VKZG_NORM_EARLY_US");
    const bool early = !(ee && atoi(ee) == 0);
    const uint64_t early_ticks = 100ull * (uint64_t)(eu ? std::max(1, atoi(eu)) : 2000);
    // (per-kernel timing keeps the late launch: the finish's events would count the host's wait)
    NormGo go;
    const bool early_now = early && !ctx->timing;
    DevBuf& cnt = ctx->ws[WS_NORM_CNT];  // word 0: the prep's arrival counter; word 16: the sparse commits' (msm.hip k_sparse_count_scan); bytes [128, 200): the relay
    if (cnt.p == nullptr) {
        VK_TRY(cnt.ensure(256));
        VK_CHECK_HIP(hipMemsetAsync(cnt.p, 0, 256, ctx->stream));
    }
    if (early_now) {
        *hgo = 0;
        go.relay = reinterpret_cast<uint64_t*>(cnt.as<uint8_t>() + 128);
        go.flag = reinterpret_cast<const uint32_t*>(dbase + go_off);
        go.epoch = epoch;
        go.limit = early_ticks;
    }
    auto release_go = [&]() {
        std::atomic_thread_fence(std::memory_order_release);  // the inverses before the word that frees them
        *hgo = epoch;
    };
    // the last block's scan costs ~17 us of serial multiplies whatever nblk is; the host's trick
    // ~54 ns per block: the scan pays from ~128 blocks on (c1 / c2 rows: 88 -> 74 us of prep + gap,
    // width-4 rows 76 -> 58 us; a 256-row level 24 -> 43 us: profiles/r05/verkle/sparse_norm_vk/)
    static const size_t scan_min = getenv("VKZG_NORM_DEVSCAN") ? (size_t)atol(getenv("VKZG_NORM_DEVSCAN")) : 128;  // A/B
    if (scan_min != 0 && nblk >= scan_min) {
        // the block products scanned on the device (k_norm_prep_vk's last block): the host inverts
        // their total only; page-locked [total | its inverse | flag] in the same alternating halves
        DevBuf& dt = ctx->ws[WS_NORM_TOT];
        VK_TRY(dt.ensure(2 * nblk * sizeof(fe<F>) + nblk * F::N * 8));
        fe<F>* dtot = dt.as<fe<F>>();
        // VKZG_NORM_TAGS=0 (read per call, A/B): a fence per block before its arrival instead
        const char* te = getenv("VKZG_NORM_TAGS");
        uint64_t* tags = (te && atoi(te) == 0) ? nullptr : reinterpret_cast<uint64_t*>(dtot + 2 * nblk);
        hflags[0] = 0;
        VK_LAUNCH(ctx, "norm_prep", k_norm_prep_vk, nblk, 256, 0, static_cast<BN254G1::Acc*>(d_rows), n, add_ids,
                  add_xy, add_inf, others.as<fe<F>>(), dtot, dflags, epoch, cnt.as<uint32_t>(), dtot + nblk, dh, tags);
        static const bool dbg_on = getenv("VKZG_NORM_DEBUG") != nullptr;
        DevBuf dbgbuf(ctx);
        if (early_now && dbg_on) {
            VK_TRY(dbgbuf.ensure(nblk * 24));
            go.dbg = dbgbuf.as<uint64_t>();
        }
        if (early_now) {
            go.per_block = 0;
            go.prod = dh;
            go.inv = dh + 1;
            VK_LAUNCH(ctx, "norm_finish", k_norm_finish_vk, nblk, 256, 0, static_cast<const BN254G1::Acc*>(d_rows), n,
                      others.as<fe<F>>(), dtot + nblk, dst, out_xy, out_inf, out_item, (const fe<F>*)nullptr, go);
        }
        const auto d0 = std::chrono::steady_clock::now();
        if (overlap && *overlap) (*overlap)();
        bool seen = false;
        const auto w0 = std::chrono::steady_clock::now();
        for (uint32_t spins = 0;; spins++) {
            if (hflags[0] == epoch) {
                seen = true;
                break;
            }
            if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - w0 > std::chrono::milliseconds(20)) break;
            _mm_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        // (queued early: this wait also covers the finish, whose blocks invert on their own past their bound)
        if (!seen) VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        h[1] = fe_inv_bin<F>(h[0]);  // never zero: identities count as 1
        const auto d1 = std::chrono::steady_clock::now();
        if (early_now) release_go();
        static const bool dbg = getenv("VKZG_NORM_DEBUG") != nullptr;
        if (dbg)
            fprintf(stderr, "[norm] n %zu nblk %zu early %d overlap %.1f us, flag wait + inverse %.1f us\n", n, nblk,
                    (int)early_now, std::chrono::duration<double, std::micro>(w0 - d0).count(),
                    std::chrono::duration<double, std::micro>(d1 - w0).count());
        if (early_now) {
            if (go.dbg) {
                const auto g0 = std::chrono::steady_clock::now();
                VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
                const double sync_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g0).count();
                std::vector<uint64_t> hd(nblk * 3);
                VK_CHECK_HIP(hipMemcpy(hd.data(), go.dbg, nblk * 24, hipMemcpyDeviceToHost));
                uint64_t tmin = ~0ull, e0 = hd[1], emax = 0, smin = ~0ull, smax = 0;
                size_t timed_out = 0;
                for (size_t b = 0; b < nblk; b++) {
                    tmin = std::min(tmin, hd[3 * b]);
                    smin = std::min(smin, hd[3 * b]);
                    smax = std::max(smax, hd[3 * b]);
                    emax = std::max(emax, hd[3 * b + 1]);
                    timed_out += hd[3 * b + 2] == 0;
                }
                fprintf(stderr, "[norm go] block 0 waited %.1f us (seen %d); starts span %.1f us; last block done waiting %.1f us after block 0; %zu timed out; host sync after go %.1f us\n",
                        (hd[1] - hd[0]) / 100.0, (int)hd[2], (smax - smin) / 100.0, ((double)emax - (double)e0) / 100.0,
                        timed_out, sync_us);
            }
            return VC_OK;
        }
        std::atomic_thread_fence(std::memory_order_release);  // the inverse before the launch that reads it
        VK_LAUNCH(ctx, "norm_finish", k_norm_finish_vk, nblk, 256, 0, static_cast<const BN254G1::Acc*>(d_rows), n,
                  others.as<fe<F>>(), dtot + nblk, dst, out_xy, out_inf, out_item, dh + 1, NormGo{});
        return VC_OK;
    }
    for (size_t b = 0; b < nblk; b++) hflags[b] = 0;
    VK_LAUNCH(ctx, "norm_prep", k_norm_prep_vk, nblk, 256, 0, static_cast<BN254G1::Acc*>(d_rows), n, add_ids, add_xy,
              add_inf, others.as<fe<F>>(), dh, dflags, epoch, (uint32_t*)nullptr, (fe<F>*)nullptr, (fe<F>*)nullptr,
              (uint64_t*)nullptr);
    if (early_now) {
        go.per_block = 1;
        go.prod = dh;
        go.inv = dh + nblk;
        VK_LAUNCH(ctx, "norm_finish", k_norm_finish_vk, nblk, 256, 0, static_cast<const BN254G1::Acc*>(d_rows), n,
                  others.as<fe<F>>(), dh + nblk, dst, out_xy, out_inf, out_item, (const fe<F>*)nullptr, go);
    }
    if (overlap && *overlap) (*overlap)();
    // Montgomery's trick over the block products: the forward products are taken as the blocks'
    // flags arrive (blocks finish roughly in order), so only the inversion and the backward pass
    // follow the last block
    fe<F>* inv = h + nblk;
    size_t done = 0;  // blocks [0, done) seen and multiplied in
    auto take = [&](size_t upto) {
        for (; done < upto; done++) inv[done] = done ? fe_mul<F>(inv[done - 1], h[done]) : h[done];
    };
    bool seen = false;
    const auto w0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 0;; spins++) {
        size_t b = done;
        while (b < nblk && hflags[b] == epoch) b++;
        if (b > done) {
            std::atomic_thread_fence(std::memory_order_acquire);  // the products after their flags
            take(b);
        }
        if (done == nblk) {
            seen = true;
            break;
        }
        if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - w0 > std::chrono::milliseconds(20)) break;
        _mm_pause();
    }
    if (!seen) {
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        take(nblk);
    }
    fe<F> run = fe_inv_bin<F>(inv[nblk - 1]);
    for (size_t b = nblk - 1; b > 0; b--) {
        const fe<F> ib = fe_mul<F>(run, inv[b - 1]);
        run = fe_mul<F>(run, h[b]);
        inv[b] = ib;
    }
    inv[0] = run;
    if (early_now) {
        release_go();
        return VC_OK;
    }
    std::atomic_thread_fence(std::memory_order_release);  // the inverses before the launch that reads them
    VK_LAUNCH(ctx, "norm_finish", k_norm_finish_vk, nblk, 256, 0, static_cast<const BN254G1::Acc*>(d_rows), n,
              others.as<fe<F>>(), dh + nblk, dst, out_xy, out_inf, out_item, (const fe<F>*)nullptr, NormGo{});
    return VC_OK;
}

// normalise n device accumulators to canonical affine (device outputs)
int normalize_to_canon(vc_ctx* ctx, int curve, const void* d_acc, size_t n, void* d_out_xy, uint8_t* d_out_inf) {
    if (n == 0) return VC_OK;
#define VK_NORM_(C)                                                                                      \
    normalize_split<C>(ctx, reinterpret_cast<const C::Acc*>(d_acc), n, (C::Aff*)nullptr,                \
                       reinterpret_cast<uint32_t*>(d_out_xy), d_out_inf)
    switch (curve) {
        case VC_CURVE_BN254: return VK_NORM_(BN254G1);
        case VC_CURVE_BLS12_381: return VK_NORM_(BLS381G1);
        case VC_CURVE_BANDERSNATCH: return VK_NORM_(Bandersnatch);
    }
#undef VK_NORM_
    return VC_E_INVALID;
}

template <class C>
static int lead_table_t(vc_ctx* ctx, Table* t, int k, int c, Table** out) {
    using Aff = typename C::Aff;
    *out = nullptr;
    if (k <= 0 || (size_t)k > t->n) return VC_E_INVALID;
    if (t->lead && t->lead_k == k && t->lead_c == c) {
        *out = t->lead;
        return VC_OK;
    }
    delete t->lead;
    t->lead = nullptr;
    // only where it leaves the device 4 GB free (as the first-use tables, fb_default_c): otherwise
    // no lead table and the caller keeps t; it then counts in the context's fb_auto_used()
    {
        using Fr = FrOf<C>;
        const size_t W = (size_t)(Fr::BITS + 1 + c - 1) / c;
        const double bytes = (double)k * (double)(W << (c - 1)) * (double)sizeof(FbE<C>);
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && bytes > (double)free_b - 4e9) return VC_OK;
    }
    Table* s = new Table();
    s->curve = t->curve;
    s->n = (size_t)k;
    s->subgroup = t->subgroup;
    int st = s->bases.ensure((size_t)k * sizeof(Aff));
    if (st == VC_OK) st = s->inf.ensure((size_t)k);
    if (st == VC_OK && (hipMemcpyAsync(s->bases.p, t->bases.p, (size_t)k * sizeof(Aff), hipMemcpyDeviceToDevice,
                                       ctx->stream) != hipSuccess ||
                        hipMemcpyAsync(s->inf.p, t->inf.p, (size_t)k, hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess))
        st = VC_E_HIP;
    if (st == VC_OK) st = fixed_base_precompute(ctx, s, c);
    if (st != VC_OK) {
        delete s;
        (void)hipGetLastError();
        return st == VC_E_OOM ? VC_OK : st;  // out of memory: no lead table, the caller keeps t
    }
    t->lead = s;
    t->lead_k = k;
    t->lead_c = c;
    *out = s;
    return VC_OK;
}
int lead_table(vc_ctx* ctx, Table* t, int k, int c, Table** out) {
    switch (t->curve) {
        case VC_CURVE_BN254: return lead_table_t<BN254G1>(ctx, t, k, c, out);
        case VC_CURVE_BLS12_381: return lead_table_t<BLS381G1>(ctx, t, k, c, out);
        case VC_CURVE_BANDERSNATCH: return lead_table_t<Bandersnatch>(ctx, t, k, c, out);
    }
    *out = nullptr;
    return VC_E_INVALID;
}

int fixed_base_precompute(vc_ctx* ctx, Table* t, int c, int windows) {
    switch (t->curve) {
        case VC_CURVE_BN254: return fb_precompute_t<BN254G1>(ctx, t, c, windows);
        case VC_CURVE_BLS12_381: return fb_precompute_t<BLS381G1>(ctx, t, c, windows);
        case VC_CURVE_BANDERSNATCH: return fb_precompute_t<Bandersnatch>(ctx, t, c, windows);
    }
    return VC_E_INVALID;
}

bool fb_small_path(vc_ctx* ctx, Table* t, size_t width, size_t batch) {
    if (t->curve != ctx->curve || batch == 0 || batch > 64) return false;
    if (!ctx->fb_lanes) {
        switch (t->curve) {
            case VC_CURVE_BN254: ctx->fb_lanes = resident_lanes(k_fb_commit_cm<BN254G1, BN254Fr>, 256); break;
            case VC_CURVE_BLS12_381: ctx->fb_lanes = resident_lanes(k_fb_commit_cm<BLS381G1, BLS381Fr>, 256); break;
            default: ctx->fb_lanes = resident_lanes(k_fb_commit_cm<Bandersnatch, BandFr>, 256); break;
        }
    }
    const size_t lanes = ctx->fb_lanes ? ctx->fb_lanes : 131072;
    size_t W = (size_t)t->fb_W;
    if (!t->fb_c) {  // before the default tables exist: the geometry fb_commit_t will build
        int c = 8, bits = 255;
        switch (t->curve) {
            case VC_CURVE_BN254: c = fb_default_c<BN254Fr>(t->n, ctx->fb_auto_used()), bits = BN254Fr::BITS; break;
            case VC_CURVE_BLS12_381: c = fb_default_c<BLS381Fr>(t->n, ctx->fb_auto_used()), bits = BLS381Fr::BITS; break;
            default: c = fb_default_c<BandFr>(t->n, ctx->fb_auto_used()), bits = BandFr::BITS; break;
        }
        W = (size_t)(bits + 1 + c - 1) / c;
    }
    return batch * width * W <= lanes;
}

int msm_batch_run(vc_ctx* ctx, Table* t, size_t width, const void* d_sc, size_t batch, int mont,
                  void* d_out_xy, uint8_t* d_out_inf, uint64_t* h_out_xy, uint8_t* h_out_inf, bool* on_host,
                  const PinBuf* pin_sc, const std::function<void()>* overlap, const StrideCols* with_cols,
                  const IpaRows* ipa) {
    bool dummy = false;
    if (!on_host) on_host = &dummy;
    *on_host = false;
    if (h_out_xy && !h_out_inf) return VC_E_INVALID;
    switch (t->curve) {
        case VC_CURVE_BN254:
            return fb_commit_t<BN254G1, BN254Fr>(ctx, t, width, d_sc, batch, mont, d_out_xy, d_out_inf, h_out_xy,
                                                 h_out_inf, on_host, pin_sc, overlap, with_cols, ipa);
        case VC_CURVE_BLS12_381:
            return fb_commit_t<BLS381G1, BLS381Fr>(ctx, t, width, d_sc, batch, mont, d_out_xy, d_out_inf, h_out_xy,
                                                   h_out_inf, on_host, pin_sc, overlap, with_cols, ipa);
        case VC_CURVE_BANDERSNATCH:
            return fb_commit_t<Bandersnatch, BandFr>(ctx, t, width, d_sc, batch, mont, d_out_xy, d_out_inf, h_out_xy,
                                                     h_out_inf, on_host, pin_sc, overlap, with_cols, ipa);
    }
    return VC_E_INVALID;
}

}  // namespace vk
