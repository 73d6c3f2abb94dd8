#!/bin/bash
# round-3 probe batch 21: marginal form of the tail's bit stage (VKZG_TAIL_MARGINAL A/B)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3z}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_comm.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py > $O/tests_full.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
for k in 1 2; do
for m in 0 1; do
VKZG_TAIL_MARGINAL=$m timeout -k 10 120 python -u $P bls12_381 20 > $O/radix_m${m}_$k.txt 2>&1 || exit 1
done
done
for m in 0 1; do
VKZG_TAIL_MARGINAL=$m VKZG_MSM_SHARED=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/vb_m$m.txt 2>&1 || exit 1
VKZG_TAIL_MARGINAL=$m timeout -k 10 120 python -u $P bn254 20 > $O/bn254_m$m.txt 2>&1 || exit 1
VKZG_TAIL_MARGINAL=$m timeout -k 10 200 python -u verkle-kzg_amd/tools/scale_probe.py > $O/scale_m$m.txt 2>&1 || exit 1
VKZG_TAIL_MARGINAL=$m timeout -k 10 120 python -u verkle-kzg_amd/tools/kzg_trace.py fused > $O/kzg_m$m.txt 2>&1 || exit 1
done
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
