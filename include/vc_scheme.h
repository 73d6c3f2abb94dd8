/* vc_scheme.h -- scheme-level C ABI of libvkzg.so: the reference's VectorCommitment
 * operations (/root/reference/vector-commit/src/lib.rs:70-174) for BN254 G1, with every
 * MSM / quotient / fold on the GPU and the serial Fiat-Shamir work on the host.
 *
 * Field elements (Fr) are 4 canonical little-endian u64 limbs; points are canonical affine
 * x[4], y[4] + a u8 identity flag (as in vc_msm.h).  All calls are synchronous and return
 * VC_OK or a VC_E_* status (vc_msm.h).  The reference's `todo!()` batch methods
 * (prove_batch / verify_batch, ipa/mod.rs:156-189, kzg/mod.rs:156-197) have no counterpart.
 *
 * Scope: the protocol layer is instantiated for BN254 (the only curve the reference runs,
 * vector-commit/Cargo.toml:15).  The MSM / commit engines (vc_msm.h) also serve BLS12-381 G1
 * and Bandersnatch.
 */
#ifndef VC_SCHEME_H
#define VC_SCHEME_H

#include <stddef.h>
#include <stdint.h>

#include "vc_msm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- Fiat-Shamir (a12)
 * TranscriptHasher (transcript.rs:28-62): append(label || compressed(value)); digest(label) =
 * hash_to_field(state || label) with DefaultFieldHasher<Sha256> and DST = the label given at
 * creation; then state = ser(out) || label. */
typedef struct vc_transcript vc_transcript;
vc_transcript* vc_transcript_new(const char* label);
/* which SHA-256 rounds the host transcript runs on this machine: 1 = x86 SHA extensions (SHA-NI),
 * 0 = the portable rounds (same digests; a machine-dependent speed, reported by bench.py) */
int vc_host_sha256_path(void);
vc_transcript* vc_transcript_clone(const vc_transcript* t);
void vc_transcript_free(vc_transcript* t);
void vc_transcript_reserve(vc_transcript* t, size_t bytes); /* capacity hint for long transcripts */
int vc_transcript_append_bytes(vc_transcript* t, const uint8_t* bytes, size_t n, const char* label);
int vc_transcript_append_point(vc_transcript* t, const uint64_t* xy, uint8_t inf, const char* label);
int vc_transcript_append_fr(vc_transcript* t, const uint64_t* fr, const char* label);
int vc_transcript_append_u64(vc_transcript* t, uint64_t v, const char* label);
int vc_transcript_digest(vc_transcript* t, const char* label, uint64_t* out_fr);
/* raw hash_to_field(msg) mod r with the given DST */
int vc_hash_to_field(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dst_len, uint64_t* out_fr);

/* ---------------------------------------------------------------- serialisation (a13)
 * arkworks 0.4 compressed SW encoding (32 B) and VCCommitment::to_data_item (lib.rs:56-67). */
int vc_point_compress(const uint64_t* xy, uint8_t inf, uint8_t* out32);
/* batched on the device: n points -> n Fr (canonical) */
int vc_to_data_item_batch(vc_ctx* ctx, const uint64_t* xy, const uint8_t* inf, size_t n, uint64_t* out_fr);

/* ---------------------------------------------------------------- CRS (a15)
 * IPAPointGenerator::gen (ipa_point_generator.rs:51-67): first `num` accepted points of
 * sha256(seed || le64(i)) -> Affine::from_random_bytes.  VC_E_RANGE if num > max
 * (PointGeneratorError::OutOfBounds, Appendix B.1). */
int vc_ipa_crs(const uint8_t* seed, size_t seed_len, size_t max, size_t num, uint64_t* out_xy);
/* KZG::setup (kzg/mod.rs:115-124): Lagrange SRS L_j = l_j(s) * G over the domain of size
 * n = next_pow2(max_items), computed on the device; out n points (table uploaded into ctx). */
int vc_kzg_setup(vc_ctx* ctx, size_t max_items, const uint64_t* secret_fr, int* table_id, size_t* size);

/* ---------------------------------------------------------------- IPA (ipa/mod.rs)
 * `table` holds the N + 1 CRS points g[0..N], q (IPAUniversalParams::new_from_vec).
 * Proof layout: L[k], R[k] points (k = log2 N rounds), tip, y. */
typedef struct {
    size_t rounds;
    uint64_t* l_xy; uint8_t* l_inf;   /* rounds x 8 u64, rounds */
    uint64_t* r_xy; uint8_t* r_inf;
    uint64_t tip[4];
    uint64_t y[4];
} vc_ipa_proof;

int vc_ipa_commit(vc_ctx* ctx, int table, size_t N, const uint64_t* data, size_t batch,
                  uint64_t* out_xy, uint8_t* out_inf);
/* prove_point (:137-154 -> low_level_ipa :268-319). transcript may be NULL (fresh "ipa").
 * Proves `batch` independent openings at once (same N, one CRS): data batch x N, points batch,
 * commitments batch; transcripts NULL or an array of batch handles (consumed state). */
int vc_ipa_prove(vc_ctx* ctx, int table, size_t N, const uint64_t* data, const uint64_t* com_xy,
                 const uint8_t* com_inf, const uint64_t* points, size_t batch,
                 vc_transcript** transcripts, vc_ipa_proof* proofs);
/* verify_point (:165-181 -> low_level_verify_ipa :321-360); result 1 = valid, 0 = invalid */
int vc_ipa_verify(vc_ctx* ctx, int table, size_t N, const uint64_t* com_xy, uint8_t com_inf,
                  const uint64_t* point, const vc_ipa_proof* proof, vc_transcript* transcript,
                  int* result);
/* prove_commitment (:199-234): proof of knowledge of the first n = data.max() + 1 values
 * behind a commitment (L, R per round, tip; y is set to 0). n must be a power of two: the
 * reference's assert in vec_add_and_distribute (utils.rs:37) panics on any odd split above 1
 * -> VC_E_INVALID here. Fresh "ipa" transcript, `batch` proofs of the same n at once. */
int vc_ipa_prove_commitment(vc_ctx* ctx, int table, size_t n, const uint64_t* data, const uint64_t* com_xy,
                            const uint8_t* com_inf, size_t batch, vc_ipa_proof* proofs);
/* verify_commitment_proof (:237-265) over g[0..2^rounds]; result 1 = valid, 0 = invalid */
int vc_ipa_verify_commitment_proof(vc_ctx* ctx, int table, const uint64_t* com_xy, uint8_t com_inf,
                                   const vc_ipa_proof* proof, int* result);

/* ---------------------------------------------------------------- KZG (kzg/mod.rs)
 * prove_point (:136-154): y = evaluate(point), q = divide_by_vanishing(index) when
 * point <= size, else divide_by_vanishing_outside_domain(point); proof = MSM(L, q).
 * evals may be shorter than the domain (`max`); VC_E_DOMAIN for point == size (the
 * reference panics there, Appendix B.4). */
int vc_kzg_prove(vc_ctx* ctx, int table, size_t size, const uint64_t* evals, size_t max,
                 const uint64_t* point, uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y);
/* same with the evaluations already in device memory (canonical, 4 u64 each) */
int vc_kzg_prove_device(vc_ctx* ctx, int table, size_t size, const void* d_evals, size_t max,
                        const uint64_t* point, uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y);
/* commit + prove_point in one call (configs[3]'s unit): C = commit(evals) (kzg/mod.rs:126-134) and
 * the proof at `point` as vc_kzg_prove_device; both MSMs over the SRS run as one batched
 * pipeline (vc_msm_device_many). */
int vc_kzg_commit_prove_device(vc_ctx* ctx, int table, size_t size, const void* d_evals, size_t max,
                               const uint64_t* point, uint64_t* com_xy, uint8_t* com_inf, uint64_t* proof_xy,
                               uint8_t* proof_inf, uint64_t* y);
/* multi-GPU open: the quotient (every part computes it; it is elementwise and ~10 % of the
 * MSM) and window slice `part` of `parts` of the proof MSM as an un-normalised accumulator;
 * the parts' accumulators sum (vc_partials_sum) to the proof */
int vc_kzg_prove_device_part(vc_ctx* ctx, int table, size_t size, const void* d_evals, size_t max,
                             const uint64_t* point, int part, int parts, uint32_t* out_acc, uint64_t* y);
/* KZG::prove_all_points (kzg/mod.rs:200-235), the FK amortised opening -- private and never
 * called in the reference (its test at :299 has no #[test]). table = the Lagrange SRS of domain
 * `size`; evals = n_evals values (the data's own domain is next_pow2(n_evals), as
 * LagrangeBasis::from_vec). Outputs *count points (out_xy, out_inf) and values (out_y = data[i]).
 *   mode 0: the reference's computation exactly -- coefficients c of the data's interpolant of
 *     degree d, c_hat = [c_d, 0^(d+1), c_0 .. c_{d-1}] cut to the domain D::new(2 d), g1 =
 *     ifft(lagrange SRS) over the key domain, s_hat = reverse(g1[0..d]) || 0, h_hat =
 *     ifft(fft(s_hat) .* fft(c_hat)); returns (h_hat[i], data[i]) for i < that domain.
 *     VC_E_DOMAIN where the reference panics: all-zero data (coeffs[degree] of an empty
 *     polynomial), a domain larger than the data (data[i] out of bounds), d > size.
 *   mode 1: the opening proofs FK computes (what the reference's test expects): for every i <
 *     size, pi_i = [q_i(s)]_1 with q_i = (f - f(w^i)) / (X - w^i) -- the Toeplitz product of the
 *     coefficients with the monomial SRS fft(lagrange SRS) by a 2 size circulant, then an FFT.
 *     Equal to vc_kzg_prove at index i; n_evals <= size (VC_E_RANGE otherwise).
 * out_xy: count x 2 NL u64 (count <= size, or the mode-0 domain); out_y: count x 4 u64. */
int vc_kzg_prove_all_points(vc_ctx* ctx, int table, size_t size, const uint64_t* evals, size_t n_evals, int mode,
                            uint64_t* out_xy, uint8_t* out_inf, uint64_t* out_y, size_t* count);
/* the quotient alone (a5/a6), for parity tests: q (size x 4 u64) and y */
int vc_kzg_quotient(vc_ctx* ctx, size_t size, const uint64_t* evals, size_t max, const uint64_t* point,
                    uint64_t* q_out, uint64_t* y);

/* ---------------------------------------------------------------- multiproof (multiproof.rs)
 * scheme: 0 = IPA (table = N + 1 CRS points), 1 = KZG (table = Lagrange SRS of size N).
 * queries: data Q x N (Fr), commitments Q, z Q (u64, < N), y Q (Fr).
 * Output: proof D and the inner proof (IPA proof or KZG (proof point, y)). */
int vc_multiproof_prove(vc_ctx* ctx, int scheme, int table, size_t N, size_t Q, const uint64_t* data,
                        const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z,
                        const uint64_t* y, uint64_t* d_xy, uint8_t* d_inf, vc_ipa_proof* ipa_proof,
                        uint64_t* kzg_proof_xy, uint8_t* kzg_proof_inf, uint64_t* kzg_y);
/* The same prover in three phases, so the Q x N field phase shards over GPUs with one
 * exchange. vc_multiproof_prove == begin + accumulate(all Q) + finish(G=1).
 * phase 1 (host, every rank): transcript over all (C, z, y) (:106-114), challenge r
 *   (canonical), and the number of distinct query points `rows` (the rows of S). Pure host code,
 *   safe to call from several threads at once: above 4096 queries each call runs one filler
 *   thread of its own beside its SHA-256 (not the shared host pool), so concurrent transcripts
 *   proceed side by side. */
int vc_multiproof_begin(size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z,
                        const uint64_t* y, vc_transcript** transcript, uint64_t* r, size_t* rows);
/* phase 2 (device, per shard): S[row][k] = sum r^i f_i[k] over queries i in [first, first + Qs)
 *   grouped by point; d_data = that slice's Qs x N evaluations (canonical, device); d_S =
 *   rows x N x 4 u64 (canonical, device). z = ALL Q points (it fixes the rows). */
int vc_multiproof_accumulate(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* z, size_t first, size_t Qs,
                             const void* d_data, const uint64_t* r, void* d_S);
/* phases 1 + 2 in one call, the host transcript on a helper thread while the calling thread sorts
 *   this shard's queries by point and uploads the plan (only the per-point sums wait for r): the
 *   same transcript, r and S as vc_multiproof_begin + vc_multiproof_accumulate. rows (the size of
 *   d_S) from vc_multiproof_rows. On error no transcript is returned. */
int vc_multiproof_rows(size_t N, size_t Q, const uint64_t* z, size_t* rows);
int vc_multiproof_begin_accumulate(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf,
                                   const uint64_t* z, const uint64_t* y, size_t first, size_t Qs, const void* d_data,
                                   void* d_S, vc_transcript** transcript, uint64_t* r);
/* phase 3: G shards' S matrices (device, contiguous, e.g. an all-gather) are summed; then
 *   quotients, g, D, t, h, E and the inner proof (:129-175). Advances `transcript`. */
int vc_multiproof_finish(vc_ctx* ctx, int scheme, int table, size_t N, size_t Q, const uint64_t* z,
                         const void* d_S_parts, int G, vc_transcript* transcript, uint64_t* d_xy, uint8_t* d_inf,
                         vc_ipa_proof* ipa_proof, uint64_t* kzg_proof_xy, uint8_t* kzg_proof_inf, uint64_t* kzg_y);
/* Proof-parallel: P independent multiproofs of Q queries each on one GPU (a caller proving
 * several blocks). Per proof the result is vc_multiproof_prove's; the host transcripts run on
 * worker threads beside the GPU's per-point sums, and the D / E commits and (IPA) the inner
 * proofs run once for all P proofs (batched). Layouts: com_xy [P][Q][8], com_inf [P][Q],
 * z [P][Q], y [P][Q][4] (host); d_data [P][Q][N] x 4 u64 canonical (device); outputs d_xy [P][8],
 * d_inf [P], and ipa_proofs[P] (scheme 0, each with caller-owned round arrays) or
 * kzg_xy [P][8], kzg_inf [P], kzg_y [P][4] (scheme 1). */
int vc_multiproof_prove_many(vc_ctx* ctx, int scheme, int table, size_t N, size_t Q, size_t P, const void* d_data,
                             const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z, const uint64_t* y,
                             uint64_t* d_xy, uint8_t* d_inf, vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy,
                             uint8_t* kzg_inf, uint64_t* kzg_y);
/* IPA-scheme verification (verify_multiproof :178-215 + low_level_verify_ipa) */
int vc_multiproof_verify_ipa(vc_ctx* ctx, int table, size_t N, size_t Q, const uint64_t* com_xy,
                             const uint8_t* com_inf, const uint64_t* z, const uint64_t* y,
                             const uint64_t* d_xy, uint8_t d_inf, const vc_ipa_proof* proof, int* result);
/* KZG-scheme: the (commitment E - D, t) pair verify_point would check with pairings
 * (out of scope); returned so a caller can run its own pairing check. */
int vc_multiproof_kzg_claim(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf,
                            const uint64_t* z, const uint64_t* y, const uint64_t* d_xy, uint8_t d_inf,
                            uint64_t* c_xy, uint8_t* c_inf, uint64_t* t);

#ifdef __cplusplus
}
#endif
#endif /* VC_SCHEME_H */
