/* vc_verkle.h -- verkle-tree commitments over libvkzg.so.
 *
 * Mirrors /root/reference/verkle-tree/src: VerkleTree<N, u8, VC, U256> (lib.rs:85-138) and
 * Node (node.rs:35-277): Internal / Extension nodes, insert (node.rs:133-204), get
 * (node.rs:74-95, lib.rs:119-125), path_to_stem (node.rs:97-120) and gen_commitment
 * (node.rs:205-277). Keys are N units of u8 (the reference tests' KEY_DATA_TYPE); values are
 * 32-byte U256 split into two Fr halves (low = bytes 0..16, high = bytes 16..32, LE, as the
 * tests' SplittableValue, lib.rs:186-194).
 *
 * The commitment is computed level by level: every dirty extension node of the tree goes
 * into one batched width-N commit (c1, c2), one batched to_data_item and one batched
 * width-4 commit; then every dirty internal node of one depth goes into one batched
 * width-256 commit, deepest level first -- instead of the reference's one recursive commit
 * per node. Rows are sparse: an internal node has a few non-zero children of 256, so only
 * non-zeros are expanded into table points. The commitment scheme is whatever `table` holds:
 * the KZG Lagrange SRS (vc_kzg_setup) or an IPA CRS (vc_bases_upload), BN254 G1.
 *
 * Device residency (vc_verkle_commitment, one context): every node's commitment, identity flag
 * and to_data_item live in a device mirror between calls (indexed by node id), so a level's
 * rows read their children's items there and nothing returns to the host but the root; the
 * host sends only the extension leaf values and each level's (column, child id) lists. An
 * updated internal node whose last commitment is in the mirror is recommitted as a delta row,
 * C_old + sum over the slots changed since of (item(new child) - item(old child)) L_slot (the
 * slots are logged at insert time) -- the same group element as its full row. A call that
 * fails leaves every dirty node to be recommitted in full by the next one. VKZG_VERKLE_DEV=0
 * (read per call) takes the host-built path the sharded / group commitments use.
 *
 * Reference quirks kept: the extension commit width is the key length
 * N, not 256; the stem keeps the key's last unit; internal nodes commit at width 256;
 * a key that differs from an existing extension's stem only in the last unit makes the
 * reference panic ("Traversed to extension node with differing stem") -- here insert
 * returns VC_E_INVALID and leaves the tree unchanged. */
#ifndef VC_VERKLE_H
#define VC_VERKLE_H
#include <stddef.h>
#include <stdint.h>

#include "vc_msm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vc_verkle vc_verkle;

/* VerkleTree::new (lib.rs:104-110); key_len = N (2..32 units of u8) */
vc_verkle* vc_verkle_new(int key_len);
void vc_verkle_free(vc_verkle* t);
/* insert_single (lib.rs:112-116): key = N bytes, value = 32 bytes */
int vc_verkle_insert(vc_verkle* t, const uint8_t* key, const uint8_t* value32);
/* get_single (lib.rs:118-125): *found = 0 when absent */
int vc_verkle_get(const vc_verkle* t, const uint8_t* key, uint8_t* value32, int* found);
/* path_to_stem (lib.rs:131-137): up to max_len entries of (prefix length, unit); *len set;
 * VC_E_INVALID for the reference's InvalidPath */
int vc_verkle_path(const vc_verkle* t, const uint8_t* key, size_t max_len, uint8_t* units, size_t* len);
/* commitment (lib.rs:127-129): root commitment, canonical affine BN254 G1 (x, y: 4 u64 each) */
int vc_verkle_commitment(vc_ctx* ctx, int table, vc_verkle* t, uint64_t* out_xy, uint8_t* out_inf);
/* diagnostics: per node id (up to max) its type (0 internal, 1 extension), level and committed
 * to_data_item (4 u64, canonical); *n = the node count */
int vc_verkle_debug_nodes(vc_verkle* t, size_t max, uint8_t* type, int32_t* level, uint64_t* items, size_t* n);
/* diagnostics (no GPU): the device path's extension host stage -- c1 / c2 rows of every
 * extension node built and merged into one buffer -- run `reps` times; *us = the median (us) */
int vc_verkle_debug_ext_stage(vc_verkle* t, int reps, double* us);
/* node counts (diagnostics): internal, extension, dirty */
int vc_verkle_stats(const vc_verkle* t, size_t* internal, size_t* extension, size_t* dirty);

#ifdef __cplusplus
}
#endif
#endif /* VC_VERKLE_H */
