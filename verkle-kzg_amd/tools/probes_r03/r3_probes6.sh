#!/bin/bash
# round-3 probe batch 6: fix-up walk with a lane per owner thread vs a lane per bucket
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3l}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py > $O/tests_msm.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "radix or 2e20 or many or chunk" > $O/tests_full.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
for i in 1 2; do
timeout -k 10 120 python -u $P bls12_381 20 > $O/own$i.txt 2>&1 || exit 1
VKZG_FIXUP_OWN=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/bucket$i.txt 2>&1 || exit 1
done
VKZG_MSM_SHARED=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/varbase_own.txt 2>&1 || exit 1
VKZG_MSM_SHARED=0 VKZG_FIXUP_OWN=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/varbase_bucket.txt 2>&1 || exit 1
timeout -k 10 120 python -u verkle-kzg_amd/tools/adversarial_probe.py > $O/adversarial.txt 2>&1 || exit 1
