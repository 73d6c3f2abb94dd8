/* vc_comm.h -- multi-GPU entry points of libvkzg.so (one process or thread per GPU).
 *
 * The reference is single-process CPU code; its batch workloads are what shard across the GPUs
 * of a node: one MSM (split by Pippenger windows), batches of independent
 * commitments (verkle-tree node updates, the commit phase of multiproofs: contiguous slices), a
 * KZG opening (window-split proof MSM), and a multiproof (query slices, one exchange of the
 * per-point sums). Every entry point below runs this rank's share on its vc_ctx and ends with ONE
 * all-gather per exchange step through a vc_comm, so every rank returns the whole result.
 *
 * A vc_comm is a rank in a group of `world` ranks with an all-gather:
 *   - RCCL (xGMI inside a node): vc_comm_init_rccl, with a 128-byte id made by
 *     vc_comm_unique_id on rank 0 and handed to the other ranks by the caller (its own channel:
 *     MPI, a file, torch.distributed, a Rust channel ...). RCCL is loaded at run time
 *     (librccl.so.1); VC_E_NO_DEVICE when it is not available.
 *   - host callback: vc_comm_init_host with the caller's all-gather over host buffers (any
 *     transport; tests run G ranks as G threads of one process on one GPU this way).
 * The collective order is the same on every rank (SPMD): every rank calls the same sequence of
 * sharded entry points with the same group-wide arguments. A vc_comm is used by one host thread
 * at a time. Status codes as in vc_msm.h.
 *
 * Failures are group-wide: a rank whose share fails (out of memory, a HIP error, a bad table)
 * still enters every exchange of the step, carrying its status with its records (or in a 4-byte
 * status exchange ahead of a device all-gather), so no peer is left waiting in RCCL. Every rank
 * then returns an error: the failing rank its own status, the others VC_E_PEER. Host exchanges
 * over RCCL are staged through buffers allocated once by vc_comm_init_rccl and move in fixed
 * 1 MiB pieces, so no exchange allocates on the way in.
 */
#ifndef VC_COMM_H
#define VC_COMM_H

#include <stddef.h>
#include <stdint.h>

#include "vc_msm.h"
#include "vc_scheme.h"
#include "vc_verkle.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vc_comm vc_comm;

/* all-gather over host buffers: recv (world * bytes) receives every rank's `bytes` from send, in
 * rank order; returns 0 on success. Called once per exchange step by every rank. */
typedef int (*vc_allgather_fn)(void* user, const void* send, size_t bytes, void* recv);

#define VC_COMM_ID_BYTES 128
int vc_comm_unique_id(uint8_t id[VC_COMM_ID_BYTES]);
/* device: HIP ordinal this rank's vc_ctx objects use */
int vc_comm_init_rccl(int device, int rank, int world, const uint8_t id[VC_COMM_ID_BYTES], vc_comm** out);
int vc_comm_init_host(int rank, int world, vc_allgather_fn fn, void* user, vc_comm** out);
void vc_comm_destroy(vc_comm* comm);
int vc_comm_rank(const vc_comm* comm);
int vc_comm_world(const vc_comm* comm);
/* 1 = RCCL transport, 0 = host callback */
int vc_comm_is_rccl(const vc_comm* comm);
/* the exchange primitive itself (host buffers; ctx supplies the device and stream RCCL runs on) */
int vc_comm_allgather(vc_comm* comm, vc_ctx* ctx, const void* send, size_t bytes, void* recv);

/* ------------------------------------------------------------------ sharded workloads
 * One MSM (utils::inner_product, utils.rs:16-19) over all ranks: by default rank k computes
 * Pippenger windows [kW/G, (k+1)W/G) of all n terms (vc_msm_device_window_part); with
 * vc_comm_set_msm_split(comm, VC_COMM_SPLIT_POINTS) rank k computes the MSM of its point range
 * shard_range(n, k, G) (vc_msm_device_partial, on the table's radix window copies). One
 * all-gather of the <= 192-byte projective partials; every rank adds them. d_scalars: all n
 * scalars on this rank's device (the point split reads only its range). The split must be the
 * same on every rank. */
#define VC_COMM_SPLIT_WINDOWS 1
#define VC_COMM_SPLIT_POINTS 2
int vc_comm_set_msm_split(vc_comm* comm, int split);
int vc_msm_sharded(vc_ctx* ctx, vc_comm* comm, int table_id, size_t offset, const void* d_scalars, size_t n,
                   int mont, uint64_t* out_xy, uint8_t* out_inf);
/* Batched width-w commits (IPA::commit ipa/mod.rs:130-135, node.rs:243-271) over all ranks:
 * rank k commits the contiguous batch slice shard_range(batch, k, G) of d_scalars (all
 * batch * width scalars, device) and the slices are all-gathered into out_xy / out_inf (host,
 * all batch commitments, canonical affine). */
int vc_msm_batch_sharded(vc_ctx* ctx, vc_comm* comm, int table_id, size_t width, const void* d_scalars,
                         size_t batch, int mont, uint64_t* out_xy, uint8_t* out_inf);
/* KZG::prove_point (kzg/mod.rs:136-154) over all ranks: the quotient on every rank (elementwise)
 * and window slice k of the proof MSM; one all-gather of partials. */
int vc_kzg_prove_sharded(vc_ctx* ctx, vc_comm* comm, int table, size_t size, const void* d_evals, size_t max,
                         const uint64_t* point, uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y);
/* prove_multiproof (multiproof.rs:99-176) over all ranks, IPA (scheme 0) or KZG (scheme 1):
 * every rank hashes the transcript over all Q queries (host), accumulates the per-point sums of
 * its query slice shard_range(Q, k, G) -- d_data_slice holds that slice's Qs x N evaluations
 * (device, canonical) -- one all-gather of the sums (rows x N x 32 B), and every rank finishes
 * (quotients, D, E, inner proof). Outputs as vc_multiproof_prove. */
int vc_multiproof_prove_sharded(vc_ctx* ctx, vc_comm* comm, int scheme, int table, size_t N, size_t Q,
                                const void* d_data_slice, const uint64_t* com_xy, const uint8_t* com_inf,
                                const uint64_t* z, const uint64_t* y, uint64_t* d_xy, uint8_t* d_inf,
                                vc_ipa_proof* ipa_proof, uint64_t* kzg_proof_xy, uint8_t* kzg_proof_inf,
                                uint64_t* kzg_y);
/* Proof-parallel multiproofs over all ranks (the 8-GPU throughput mode of configs[4]): P
 * independent multiproofs of Q queries each; rank k proves proofs shard_range(P, k, G) end to end
 * (vc_multiproof_prove_many) and one all-gather of the finished proofs gives every rank all P.
 * com_xy / com_inf / z / y: all P proofs' queries (host, layouts of vc_multiproof_prove_many);
 * d_data_mine: this rank's proofs' evaluations [P_k][Q][N] (device); outputs: all P. The
 * query-sliced single multiproof (vc_multiproof_prove_sharded) is bounded near one GPU's time by
 * the transcript and finish every rank repeats (at most ~1.15x on 8 GPUs); this mode is not. */
int vc_multiproof_prove_many_sharded(vc_ctx* ctx, vc_comm* comm, int scheme, int table, size_t N, size_t Q, size_t P,
                                     const void* d_data_mine, const uint64_t* com_xy, const uint8_t* com_inf,
                                     const uint64_t* z, const uint64_t* y, uint64_t* d_xy, uint8_t* d_inf,
                                     vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy, uint8_t* kzg_inf, uint64_t* kzg_y);
/* Its exchange alone: this rank holds proofs shard_range(P, k, G) (at their global positions in
 * the outputs) and its share's status; afterwards every rank holds all P, or every rank returns
 * an error (its own status, or VC_E_PEER). A rank whose output buffers are unusable for the P
 * proofs (NULL arrays, an IPA proof with fewer than log2 N rounds) fails like a failed share:
 * it still enters the exchange and no rank writes its outputs. scheme and N size the records and
 * must be the same on every rank. ctx may be NULL over a host-callback comm. */
int vc_multiproof_gather(vc_comm* comm, vc_ctx* ctx, int status, int scheme, size_t N, size_t P, uint64_t* d_xy,
                         uint8_t* d_inf, vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy, uint8_t* kzg_inf,
                         uint64_t* kzg_y);
/* Node::gen_commitment (node.rs:205-277) level by level over all ranks: every rank holds the same
 * tree (the same inserts); the dirty extension nodes and each depth's dirty internal nodes are cut
 * into contiguous rank slices, each rank commits its slice, and one all-gather per level gives
 * every rank every commitment (extensions: one exchange after their c1 / c2 / [1, stem, c1, c2]
 * commits, which only need the node's own values; internal levels: one exchange each, deepest
 * first, because a parent needs its children's commitments). */
int vc_verkle_commitment_sharded(vc_ctx* ctx, vc_comm* comm, int table, vc_verkle* tree, uint64_t* out_xy,
                                 uint8_t* out_inf);

#ifdef __cplusplus
}
#endif
#endif /* VC_COMM_H */
