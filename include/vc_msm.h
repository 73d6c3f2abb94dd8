/* vc_msm.h -- C ABI of the MI355X vector-commitment MSM engine (libvkzg.so).
 *
 * This is the drop-in boundary for the reference's hot path. A Rust
 * `impl VectorCommitment` (reference: /root/reference/vector-commit/src/lib.rs:70-174)
 * calls these entry points over `extern "C"` in place of `utils::inner_product`
 * (vector-commit/src/utils.rs:16-19) and of the arithmetic inside `commit` /
 * `prove_point`; see INTEGRATION.md for the binding a maintainer adds.
 *
 * Conventions
 *   - All functions are synchronous at the ABI (device work is finished and, for
 *     host outputs, copied back before return) and return 0 (VC_OK) or a negative
 *     VC_E_* status; vc_strerror() names it.  Nothing here panics.
 *   - Field elements: canonical (non-Montgomery) little-endian u64 limbs.
 *     BN254 Fq / all scalar fields / Bandersnatch Fq: 4 limbs; BLS12-381 Fq: 6 limbs.
 *   - Affine points: x limbs then y limbs (2*NL u64), plus one u8 per point that is 1
 *     for the identity (its x, y are ignored).  Twisted-Edwards identity is (0, 1).
 *   - Scalars: 4 u64 limbs each.  `mont` = 0: canonical and < r;  `mont` = 1:
 *     arkworks' internal Montgomery form (the engine converts on the device).
 *   - The caller owns every host buffer; a vc_ctx owns its device copies.
 *   - A vc_ctx serialises calls internally (one mutex); share it across threads freely
 *     (the reference's multiproof bound needs UniversalParams: Sync, multiproof.rs:96).
 */
#ifndef VC_MSM_H
#define VC_MSM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* curves (the reference instantiates only BN254, vector-commit/Cargo.toml:15) */
#define VC_CURVE_BN254 0        /* BN254 G1, y^2 = x^3 + 3 (ark-bn254)              */
#define VC_CURVE_BLS12_381 1    /* BLS12-381 G1, y^2 = x^3 + 4                      */
#define VC_CURVE_BANDERSNATCH 2 /* twisted Edwards a=-5 over BLS12-381 Fr           */

/* status codes */
#define VC_OK 0
#define VC_E_INVALID (-1)     /* bad argument (null pointer, size, unknown curve)  */
#define VC_E_HIP (-2)         /* HIP runtime error                                 */
#define VC_E_OOM (-3)         /* device allocation failed                          */
#define VC_E_TABLE (-4)       /* unknown / incompatible base table id              */
#define VC_E_RANGE (-5)       /* offset + n beyond the base table                  */
#define VC_E_NOT_ON_CURVE (-6)/* an uploaded base is not on the curve              */
#define VC_E_NO_DEVICE (-7)   /* no usable gfx950 device                           */
#define VC_E_DOMAIN (-8)      /* evaluation point outside what the call supports   */
#define VC_E_COMM (-9)        /* collective failed (vc_comm.h: RCCL or the callback) */
#define VC_E_PEER (-10)       /* another rank of the vc_comm failed this step (vc_comm.h) */

typedef struct vc_ctx vc_ctx;

const char* vc_strerror(int status);
int vc_version(void);
/* Diagnostics (not part of the reference boundary): measured v_mad_u64_u32 throughput of the
 * ctx's device in tera-ops/s -- the peak of the VALU roofline bench.py reports. */
int vc_device_mad_rate(vc_ctx* ctx, double* tera_per_s);

/* Context: one device, one stream. device = HIP ordinal. */
int vc_ctx_create(int curve, int device, vc_ctx** out);
void vc_ctx_destroy(vc_ctx* ctx);
int vc_ctx_curve(const vc_ctx* ctx);
/* Launch on an external stream (e.g. torch.cuda.current_stream().cuda_stream); NULL = own. */
int vc_ctx_set_stream(vc_ctx* ctx, void* hip_stream);
/* Engine knobs (per context; defaults in brackets). None changes a result, only the path:
 *   VC_OPT_MSM_SHARED_WINDOWS [1]: a GLV MSM (BLS12-381, n >= 4096) over a WHOLE table sends all
 *     windows to one bucket set through per-table window copies B^w P_i, B^w phi(P_i), each as
 *     x, y and -y in radix-2^29 limbs (168 B): one GPU, n >= 2^18: mixed radix B = 5 x 2^16, 7
 *     windows, 7 x 2n copies = 2.47 GB at n = 2^20; window slices of a multi-GPU MSM
 *     (vc_msm_device_window_part) use B = 2^16, 8 windows (2.82 GB). Built once per table on
 *     first use and kept (a fixed-base precomputation over the CRS). A table holds ONE copy
 *     layout: alternating whole-table MSMs and window-part MSMs on the same table rebuilds the
 *     copies (~0.1 s at 2^20) on every switch, so keep one table on one path.
 *     0: plain variable-base Pippenger, no copies.
 *   VC_OPT_MSM_CHUNK_POINTS [2^27]: MSMs of more points run as summed chunks of this many
 *     (keeps the u32 entry space of the bucket sort from wrapping).
 *   VC_OPT_MSM_HOST_CHUNKS [2]: vc_msm (host scalars) on the radix shared-window path copies the
 *     scalars in this many chunks (1..4) on a second stream, each chunk's sort + accumulate under
 *     the next chunk's copy, one reduction at the end; 1 = one copy, then the MSM. */
#define VC_OPT_MSM_SHARED_WINDOWS 1
#define VC_OPT_MSM_CHUNK_POINTS 2
#define VC_OPT_MSM_HOST_CHUNKS 3
int vc_ctx_set_option(vc_ctx* ctx, int option, int64_t value);
int vc_ctx_get_option(vc_ctx* ctx, int option, int64_t* value);
/* Per-kernel device timing (HIP events around each launch on the ctx stream). */
int vc_ctx_enable_timing(vc_ctx* ctx, int on);
/* name: "msm_accumulate", "msm_digits", ... ; returns total ms and launch count */
int vc_ctx_kernel_time(vc_ctx* ctx, const char* name, double* total_ms, long* launches);
int vc_ctx_reset_timing(vc_ctx* ctx);
/* With timing on, each bucket-accumulate launch also stamps the shader clock (s_memtime) against
 * the 100 MHz constant clock (s_memrealtime) around one lane's loop: the mean effective shader clock
 * (MHz) over the launches since the last reset -- the DVFS state the accumulate ran at. */
int vc_ctx_accumulate_clock(vc_ctx* ctx, double* mhz, long* launches);

/* Base tables ---------------------------------------------------------------
 * Upload n affine bases once (validated on the device: VC_E_NOT_ON_CURVE).
 * Replaces the reference's `IPAUniversalParams::g` (ipa/mod.rs:22-28) and
 * `KZGKey::lagrange_commitments` (kzg/mod.rs:28-40). */
int vc_bases_upload(vc_ctx* ctx, const uint64_t* affine_xy, const uint8_t* inf, size_t n,
                    int* table_id);
int vc_bases_count(vc_ctx* ctx, int table_id, size_t* n);
/* Synthetic bases s_i*G with s_i = H(seed, i) mod r, generated on the device (bench input
 * generation; the reference generates its CRS at setup, kzg_point_generator.rs:32-43). */
int vc_bases_random(vc_ctx* ctx, uint64_t seed, size_t n, int* table_id);
int vc_bases_download(vc_ctx* ctx, int table_id, uint64_t* affine_xy, uint8_t* inf);

/* MSM: out = sum_i scalars[i] * bases[offset + i]  (utils::inner_product, utils.rs:16-19).
 * `zip` truncation of the reference (Appendix B.9) is the caller's n. Host scalars: n <= 1024 from
 * offset 0 of a table with precomputed fixed-base windows (vc_fixed_base_precompute) runs as one
 * fixed-base commit (the latency path); large BLS12-381 MSMs copy the scalars in
 * VC_OPT_MSM_HOST_CHUNKS chunks under the previous chunk's work. Same result either way. */
int vc_msm(vc_ctx* ctx, int table_id, size_t offset, const uint64_t* scalars, size_t n, int mont,
           uint64_t* out_xy, uint8_t* out_inf);
/* Same with scalars already resident in device memory (4 u64 per scalar). */
int vc_msm_device(vc_ctx* ctx, int table_id, size_t offset, const void* d_scalars, size_t n,
                  int mont, uint64_t* out_xy, uint8_t* out_inf);
/* `count` MSMs over one base table (the first n bases, n <= its size): scalar set k at d_scalars[k]
 * (device, 4 u64 each; mont[k] as vc_msm's flag) -> out_xy[k], out_inf[k] (canonical affine).
 * Same results as count vc_msm_device calls; when they cover a whole BLS12-381 table of >= 2^18
 * points they run as ONE pipeline (one sort into count bucket sets, one accumulate, one
 * reduction), so the latency-bound tail is paid once. */
int vc_msm_device_many(vc_ctx* ctx, int table_id, const void* const* d_scalars, const int* mont, size_t n,
                       size_t count, uint64_t* out_xy, uint8_t* out_inf);
/* Partial MSM for sharding across GPUs: returns the un-normalised accumulator (projective,
 * curve-specific words, see vc_point_words) so ranks can all-gather and add. */
int vc_point_words(int curve);
int vc_msm_device_partial(vc_ctx* ctx, int table_id, size_t offset, const void* d_scalars,
                          size_t n, int mont, uint32_t* out_acc);
/* The same from host scalars (vc_msm's chunked copy: a large BLS12-381 range copies its scalars in
 * VC_OPT_MSM_HOST_CHUNKS chunks under the previous chunk's work) -- one GPU's share of a
 * point-split MSM whose scalars live in host memory (vc_group_msm, vc_msm_sharded callers). */
int vc_msm_partial(vc_ctx* ctx, int table_id, size_t offset, const uint64_t* scalars, size_t n, int mont,
                   uint32_t* out_acc);
/* Window-sliced partial MSM (the other way to shard one MSM across GPUs): part k of `parts`
 * covers Pippenger windows [k*W/parts, (k+1)*W/parts) of ALL n terms, including their 2^(c*w)
 * weights, so the parts' accumulators sum (vc_partials_sum) to the whole MSM. Each part
 * streams every base but builds and reduces only its windows' buckets: the bucket reduction,
 * which does not shrink with n, is divided by `parts` (a point split leaves it whole). */
/* c and W chosen for an n-term MSM; terms_per_point (may be NULL) = 2 when the scalars are
 * split by the GLV endomorphism (BLS12-381, n >= 4096, tables of subgroup points: 2n terms of
 * 127-bit scalars over P_i and phi(P_i), W windows of those), else 1 */
int vc_msm_windows(int curve, size_t n, int* window_bits, int* windows, int* terms_per_point);
/* Geometry the last MSM on this context actually ran (any vc_msm* entry point): windows of radix
 * radix_mul * 2^window_bits (radix_mul > 1: the mixed-radix shared windows of a one-GPU
 * whole-table GLV MSM, e.g. 5 * 2^16 with 7 windows), terms per point, and whether all windows
 * shared one bucket set through the table's window copies. Any out pointer may be NULL. */
int vc_msm_last_plan(const vc_ctx* ctx, int* window_bits, int* windows, int* terms_per_point, int* radix_mul,
                     int* shared_windows);
int vc_msm_device_window_part(vc_ctx* ctx, int table_id, size_t offset, const void* d_scalars, size_t n,
                              int mont, int part, int parts, uint32_t* out_acc);
/* Sum k partial accumulators (host) and normalise to canonical affine. */
int vc_partials_sum(int curve, const uint32_t* accs, size_t k, uint64_t* out_xy, uint8_t* out_inf);

/* Batched width-w commits against one table: out[j] = sum_i s[j*w+i] * bases[i].
 * (IPA::commit ipa/mod.rs:130-135, verkle Node::gen_commitment node.rs:243-271) */
int vc_msm_batch(vc_ctx* ctx, int table_id, size_t width, const uint64_t* scalars, size_t batch,
                 int mont, uint64_t* out_xy, uint8_t* out_inf);
int vc_msm_batch_device(vc_ctx* ctx, int table_id, size_t width, const void* d_scalars,
                        size_t batch, int mont, void* d_out_xy, uint8_t* d_out_inf);
/* Sparse batched commits (CSR): out[g] = sum_{j in [row_ptr[g], row_ptr[g+1])} s_j * bases[cols[j]].
 * row_ptr: batch + 1 offsets; cols: column (base index) per non-zero; scalars: 4 u64 per
 * non-zero. Same fixed-base tables as vc_msm_batch; the work is proportional to the non-zeros
 * (verkle internal nodes commit ~5 non-zero children of 256, node.rs:262-271). */
int vc_msm_batch_sparse(vc_ctx* ctx, int table_id, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                        const uint64_t* scalars, int mont, uint64_t* out_xy, uint8_t* out_inf);
/* Build fixed-base window tables for a table (used by vc_msm_batch*); window_bits in [4, 20]
 * (n x ceil(bits/c) x 2^(c-1) entries of 128 B, one cache line each: 223 GB for 256 Bandersnatch
 * bases at c = 20). A table that reaches a batched commit without them gets them on first use at
 * the widest c <= 16 that fits what is left of the context's 20 GB budget for such tables
 * (VKZG_FB_BUDGET_GB), at least 8: c = 16 (17.2 GB) for the first 257-point IPA CRS. */
int vc_fixed_base_precompute(vc_ctx* ctx, int table_id, int window_bits);
/* The same with `windows` signed-digit windows of window_bits or window_bits + 1 bits (the
 * last bits + 1 - window_bits * windows windows are the wider ones; window_bits in [4, 19]).
 * Sizes a table between two uniform ones: Bandersnatch window_bits 18, windows 14 is 58 GB
 * for 256 bases with the 14 windows per scalar of the 101 GB c = 19 table. windows = 0, or at
 * least the uniform count, is vc_fixed_base_precompute. VC_E_INVALID when the windows cannot
 * cover the scalar with at most one extra bit each. */
int vc_fixed_base_precompute_windows(vc_ctx* ctx, int table_id, int window_bits, int windows);
/* Geometry of a table's fixed-base tables (0s if none yet): window bits c, windows, wide windows */
int vc_fixed_base_geometry(vc_ctx* ctx, int table_id, int* window_bits, int* windows, int* wide_windows);
/* bytes of the table's fixed-base window tables in HBM (0 when none are built) */
int vc_fixed_base_table_bytes(vc_ctx* ctx, int table_id, size_t* bytes);

#ifdef __cplusplus
}
#endif
#endif /* VC_MSM_H */
