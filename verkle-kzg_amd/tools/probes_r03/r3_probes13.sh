#!/bin/bash
# round-3 probe batch 13: staged coarse scatter with 7 cursor atomics in flight
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3s}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py > $O/tests_msm.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "radix or 2e20" > $O/tests_full.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
for i in 1 2 3; do timeout -k 10 120 python -u $P bls12_381 20 > $O/rb$i.txt 2>&1 || exit 1; done
