// Internal multi-GPU plumbing shared by comm.cpp (include/vc_comm.h) and the sharded workloads.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>

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

// Node::gen_commitment level by level (verkle.cpp); sh = nullptr: the whole tree on this ctx
int verkle_commitment(vc_ctx* ctx, int table, vc_verkle* t, uint64_t* out_xy, uint8_t* out_inf, const Shard* sh);

}  // namespace vk
