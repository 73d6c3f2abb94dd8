#!/bin/bash
# round 5 step Q: host-side phases of the 2^20 MSM call (first launch, enqueue, wait, fold, affine)
set -u
O=gpurun_out/r05_q
mkdir -p $O
export TMPDIR=/tmp
VKZG_HOST_TIMING=1 timeout -k 10 150 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 > $O/host_timing.txt 2>&1 || exit $?
grep -E "msm_host|msm_affine" $O/host_timing.txt | tail -8
