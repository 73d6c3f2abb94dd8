// Host check of the bit-stage geometry chosen by msm_tail_plan (verkle-kzg_amd/csrc/msm_tail.hpp):
// prints one JSON line per geometry (the tail shapes of the MSM paths) for tests/test_tail_plan.py.
#include <cstdio>
#include "../../verkle-kzg_amd/csrc/msm_tail.hpp"
using namespace vk;

static void show(const char* name, uint32_t S, uint32_t W, uint32_t J, uint32_t nU, bool u_total) {
    const TailPlan p = msm_tail_plan(S, W, J, nU, true, u_total);
    printf("{\"name\": \"%s\", \"h\": %u, \"K\": %u, \"nb1\": %u, \"nb2\": %u, \"per_w\": %u, \"pL\": %u, "
           "\"gL\": %u, \"gH\": %u, \"slots\": %u, \"urow\": %d}\n",
           name, p.h, p.K, p.nb1, p.nb2, p.per_w, p.pL, p.gL, p.gH, p.slots, p.urow ? 1 : 0);
}

int main() {
    show("slice8", 1u << 15, 1, 15, 1, true);      // 8-way window slice: one set of 2^15 buckets, Lseg = 1
    show("radix1", 1u << 15, 1, 15, 5, false);     // one-GPU radix MSM: 2^15 segments of 5 buckets
    show("shared12", 1u << 12, 1, 12, 1, true);    // a 20000-point shared-window MSM: 2^12 buckets
    show("kzg2", 1u << 15, 2, 15, 5, false);       // the one-call KZG: two radix sets
    show("perwin8", 1u << 13, 8, 13, 4, false);    // variable base: 8 windows, segments of 4, residue U sums
    show("perwin16", 1u << 13, 16, 13, 1, false);  // BN254 / Bandersnatch 2^20: 16 windows, acc_s
    return 0;
}
