#!/bin/bash
# round-3 probe batch 5: residue-form tail (k_msm_segr + U sums) vs the acc_s segment sums
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3k}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "radix or 2e20 or many" > $O/tests_full.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py > $O/tests_msm.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
timeout -k 10 120 python -u $P bls12_381 20 > $O/resid.txt 2>&1 || exit 1
VKZG_TAIL_RESIDUE=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/segsum.txt 2>&1 || exit 1
VKZG_SEGR_QUAD=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/resid_lane.txt 2>&1 || exit 1
timeout -k 10 120 python -u $P bls12_381 20 > $O/resid2.txt 2>&1 || exit 1
VKZG_TAIL_RESIDUE=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/segsum2.txt 2>&1 || exit 1
