#!/bin/bash
# round-3 probe batch 15: verkle host staging (uninitialised vectors, parallel chunk lists)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3v}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_verkle.py tests/test_gpu_msm.py -k "verkle or sparse" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_comm.py -k "verkle" > $O/tests_comm.txt 2>&1 || exit 1
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_probe.py > $O/verkle.txt 2>&1 || exit 1
