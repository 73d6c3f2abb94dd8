#!/bin/bash
# round 5 step O: MSM tails with direct completion (final stage writes into fine-grained
# page-locked memory and flags each block; the host polls): every -m gpu test, then an alternating
# A/B of VKZG_TAIL_POLL (1 = direct, 0 = read-back copy + stream wait) on the 2^20 BLS12-381 MSM
set -u
O=gpurun_out/r05_o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_probe.sh $O VKZG_TAIL_POLL "1 0" 3 150 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 || exit $?
VKZG_HOST_TIMING=1 timeout -k 10 150 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 > $O/host_timing_poll1.txt 2>&1 || exit $?
VKZG_HOST_TIMING=1 VKZG_TAIL_POLL=0 timeout -k 10 150 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 > $O/host_timing_poll0.txt 2>&1 || exit $?
for f in $O/VKZG_TAIL_POLL_*; do echo "$f: $(grep wall $f)"; done
