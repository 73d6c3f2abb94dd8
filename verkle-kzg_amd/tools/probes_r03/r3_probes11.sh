#!/bin/bash
# round-3 probe batch 11: LDS-staged fine sort scatter
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3q}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py > $O/tests_msm.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "radix or 2e20 or many or kzg" > $O/tests_full.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
for i in 1 2; do
timeout -k 10 120 python -u $P bls12_381 20 > $O/stage$i.txt 2>&1 || exit 1
VKZG_SORT_STAGE=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/direct$i.txt 2>&1 || exit 1
done
VKZG_MSM_SHARED=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/varbase_stage.txt 2>&1 || exit 1
VKZG_MSM_SHARED=0 VKZG_SORT_STAGE=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/varbase_direct.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w_stage -o run --output-format csv -- python3 $R/$P bls12_381 20 > $O/w_stage.txt 2>&1 || exit 1
