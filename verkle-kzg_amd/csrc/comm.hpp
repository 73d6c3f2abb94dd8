// Internal multi-GPU plumbing shared by comm.cpp (include/vc_comm.h) and the sharded workloads.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>
#include <vector>

#include "../../include/vc_verkle.h"

namespace vk {

// a rank's place in a group plus the group's all-gather over host buffers: recv (world * bytes)
// receives every rank's `bytes`, in rank order
struct Shard {
    int rank = 0, world = 1;
    std::function<int(const void* send, size_t bytes, void* recv)> allgather;
};

// contiguous near-equal split of [0, n): rank k gets [n k / G, n (k + 1) / G)
inline void shard_range(size_t n, int rank, int world, size_t* lo, size_t* hi) {
    *lo = n * (size_t)rank / (size_t)world;
    *hi = n * (size_t)(rank + 1) / (size_t)world;
}

// in-process members of a vc_group (group.cpp): their contexts and member-local table ids, and
// run(f) = f(k) for every member concurrently, returning when all have finished
struct Multi {
    std::vector<vc_ctx*> ctx;
    std::vector<int> table;
    std::function<void(const std::function<void(int)>&)> run;
};

// Node::gen_commitment level by level (verkle.cpp); sh = nullptr: the whole tree on this ctx, or
// with mu every level's commits cut into member slices committed concurrently (no exchange: the
// members write into the one tree's level records directly)
int verkle_commitment(vc_ctx* ctx, int table, vc_verkle* t, uint64_t* out_xy, uint8_t* out_inf, const Shard* sh,
                      const Multi* mu = nullptr);
// KZG::prove_point split by index range (scheme.hip): share [lo, hi) of the domain uploads only
// its evaluations, phase 1 returns its partial of the one global sum (4 u64: Montgomery Fr words),
// phase 2 takes the members' total (kzg_share_sum) and returns the MSM accumulator over SRS points
// [lo, hi) and y (canonical)
struct KzgShare;
int kzg_share_begin(vc_ctx* ctx, int table, size_t size, const uint64_t* evals, size_t max, const uint64_t* point,
                    size_t lo, size_t hi, KzgShare** out, uint64_t* partial);
int kzg_share_finish(KzgShare* s, const uint64_t* total, uint32_t* out_acc, uint64_t* y);
void kzg_share_free(KzgShare* s);
int kzg_share_sum(int curve, const uint64_t* parts, int G, uint64_t* total);
int verkle_pull_host(vc_verkle* t);
int verkle_debug_ext_stage(vc_verkle* t, int reps, double* us);
// one context, every level device-resident (verkle.cpp; vc_verkle_commitment's default)
int verkle_commitment_dev(vc_ctx* ctx, int table, vc_verkle* t, uint64_t* out_xy, uint8_t* out_inf);

}  // namespace vk
