/* vc_group.h -- one process, several GPUs: the reference's callers unchanged on a whole node.
 *
 * The reference's VectorCommitment trait (vector-commit/src/lib.rs:70-174) is stateless associated
 * functions called from one process, with rayon inside prove_multiproof (multiproof.rs:119-144).
 * A vc_group owns one vc_ctx per device and one host worker thread per member, and runs every
 * call below across its members with no SPMD code on the caller's side: the host transcript
 * once, each member's share on its own device concurrently, the results combined in host memory
 * (no collective: the members share the process). SURVEY.md 8(b) `vc_ctx_create(curve,
 * num_gpus, ...)`, 8(e) partitioning.
 *
 * Conventions are vc_msm.h's: synchronous calls, host buffers owned by the caller, canonical
 * little-endian limbs, VC_OK or a VC_E_* status. A failing member makes the call return the
 * first failing member's status (after every member has finished its share). One group call
 * runs at a time (an internal mutex); members may repeat a device (tests run two members on one
 * card).
 */
#ifndef VC_GROUP_H
#define VC_GROUP_H

#include <stddef.h>
#include <stdint.h>

#include "vc_scheme.h"
#include "vc_verkle.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vc_group vc_group;

/* ndev members on devices[0..ndev) (NULL: devices 0 .. ndev-1). */
int vc_group_create(int curve, int ndev, const int* devices, vc_group** out);
void vc_group_destroy(vc_group* g);
int vc_group_size(const vc_group* g);
/* member k's context (its knobs, timing, stream); owned by the group */
vc_ctx* vc_group_member(vc_group* g, int k);
/* How device-to-device copies from member `from` to member `to` travel (the multiproof sums to
 * member 0): VC_GROUP_PEER_SAME (one device), VC_GROUP_PEER_DIRECT (peer access enabled at
 * vc_group_create: xGMI), VC_GROUP_PEER_STAGED (no peer access: HIP stages through host memory). */
#define VC_GROUP_PEER_SAME 0
#define VC_GROUP_PEER_DIRECT 1
#define VC_GROUP_PEER_STAGED 2
int vc_group_peer_path(const vc_group* g, int from, int to);

/* Tables: a group table id names one copy per member (uploaded to every member concurrently). */
int vc_group_bases_upload(vc_group* g, const uint64_t* affine_xy, const uint8_t* inf, size_t n, int* table_id);
int vc_group_bases_random(vc_group* g, uint64_t seed, size_t n, int* table_id);
int vc_group_kzg_setup(vc_group* g, size_t max_items, const uint64_t* secret_fr, int* table_id, size_t* size);
int vc_group_fixed_base_precompute(vc_group* g, int table_id, int window_bits, int windows);
/* the member-local id of a group table (for vc_* calls on vc_group_member(g, k)) */
int vc_group_member_table(const vc_group* g, int table_id, int member, int* member_table);

/* How one MSM splits over the members:
 *   VC_GROUP_SPLIT_WINDOWS: member k computes Pippenger windows [kW/G, (k+1)W/G) of all n terms
 *     (vc_msm_device_window_part) -- every member receives all n scalars;
 *   VC_GROUP_SPLIT_POINTS: member k computes the MSM of its contiguous 1/G of the points
 *     (vc_msm_device_partial) -- every member receives only its scalars;
 *   VC_GROUP_SPLIT_AUTO (default): POINTS (host scalars: the PCIe copy is split too); for
 *     vc_group_kzg_prove index ranges of the domain (the quotient split too). */
#define VC_GROUP_SPLIT_AUTO 0
#define VC_GROUP_SPLIT_WINDOWS 1
#define VC_GROUP_SPLIT_POINTS 2
int vc_group_set_msm_split(vc_group* g, int split);

/* utils::inner_product (utils.rs:16-19) over table[offset, offset + n), host scalars. */
int vc_group_msm(vc_group* g, int table_id, size_t offset, const uint64_t* scalars, size_t n, int mont,
                 uint64_t* out_xy, uint8_t* out_inf);
/* batched width-w commits (IPA::commit ipa/mod.rs:130-135 over many datasets): contiguous batch
 * slices per member. */
int vc_group_msm_batch(vc_group* g, int table_id, size_t width, const uint64_t* scalars, size_t batch, int mont,
                       uint64_t* out_xy, uint8_t* out_inf);
/* KZG::prove_point (kzg/mod.rs:136-154), same arguments as vc_kzg_prove. Default: split by index
 * range -- member k uploads only f on its 1/G of the domain, computes the quotient there and the
 * proof MSM over SRS points of that range; the in-domain q_m (outside: y) needs one exchange of G
 * field partials between the two phases. VC_GROUP_SPLIT_WINDOWS: every member the whole quotient
 * and a window slice of the MSM (vc_kzg_prove_device_part). */
int vc_group_kzg_prove(vc_group* g, int table_id, size_t size, const uint64_t* evals, size_t max,
                       const uint64_t* point, uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y);
/* prove_multiproof (multiproof.rs:99-176), arguments as vc_multiproof_prove (host data Q x N):
 * the transcript once on the host, each member the per-point sums of its query slice, the sums
 * added on member 0, which finishes (D, t, E, inner proof). */
int vc_group_multiproof_prove(vc_group* g, int scheme, int table_id, size_t N, size_t Q, const uint64_t* data,
                              const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z, const uint64_t* y,
                              uint64_t* d_xy, uint8_t* d_inf, vc_ipa_proof* ipa_proof, uint64_t* kzg_proof_xy,
                              uint8_t* kzg_proof_inf, uint64_t* kzg_y);
/* P independent multiproofs (arguments as vc_multiproof_prove_many, but data [P][Q][N] on the
 * host): member k proves its contiguous share of the P proofs end to end. */
int vc_group_multiproof_prove_many(vc_group* g, int scheme, int table_id, size_t N, size_t Q, size_t P,
                                   const uint64_t* data, const uint64_t* com_xy, const uint8_t* com_inf,
                                   const uint64_t* z, const uint64_t* y, uint64_t* d_xy, uint8_t* d_inf,
                                   vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy, uint8_t* kzg_inf, uint64_t* kzg_y);
/* Node::gen_commitment (verkle-tree/src/node.rs:205-277) on one tree: the host walks the dirty
 * nodes once; every level's commits are cut into member slices committed concurrently. */
int vc_group_verkle_commitment(vc_group* g, int table_id, vc_verkle* tree, uint64_t* out_xy, uint8_t* out_inf);

#ifdef __cplusplus
}
#endif
#endif /* VC_GROUP_H */
