#!/bin/bash
# round-3 probe batch 19: staged coarse only for long runs
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3z}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_comm.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py > $O/tests_full.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
VKZG_MSM_SHARED=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/vb.txt 2>&1 || exit 1
timeout -k 10 120 python -u $P bn254 20 > $O/bn254.txt 2>&1 || exit 1
timeout -k 10 120 python -u $P bls12_381 20 > $O/radix.txt 2>&1 || exit 1
timeout -k 10 120 python -u verkle-kzg_amd/tools/kzg_trace.py fused > $O/kzg.txt 2>&1 || exit 1
