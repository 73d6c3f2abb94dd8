#!/bin/bash
# round-3 probe batch 17: staged coarse write-out with 16 lanes per bin; two-set staging for the KZG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3x}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "radix or 2e20 or many or kzg" > $O/tests_full.txt 2>&1 || exit 1
VKZG_SORT_CSTAGE=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "many or kzg" > $O/tests_full2.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
for i in 1 2; do timeout -k 10 120 python -u $P bls12_381 20 > $O/q16_$i.txt 2>&1 || exit 1; done
K=verkle-kzg_amd/tools/kzg_trace.py
for i in 1 2; do
timeout -k 10 120 python -u $K fused > $O/kzg_default$i.txt 2>&1 || exit 1
VKZG_SORT_CSTAGE=2 timeout -k 10 120 python -u $K fused > $O/kzg_cst2_$i.txt 2>&1 || exit 1
done
