#!/bin/bash
# round-3 probe batch 9: KZG quotient without host round trips; KZG tests; fused timing + trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3o}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kzg_device.py tests/test_gpu_scheme.py tests/test_gpu_kzg_fk.py tests/test_gpu_comm.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "kzg" > $O/tests_full.txt 2>&1 || exit 1
K=verkle-kzg_amd/tools/kzg_trace.py
timeout -k 10 120 python -u $K fused > $O/fused_in.txt 2>&1 || exit 1
timeout -k 10 120 python -u $K fused_out > $O/fused_out.txt 2>&1 || exit 1
VKZG_SORT_CHUNK=4096 timeout -k 10 120 python -u $K fused > $O/chunk4096.txt 2>&1 || exit 1
VKZG_SORT_FB=6 timeout -k 10 120 python -u $K fused > $O/fb6.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/$K fused > $O/trace.txt 2>&1 || exit 1
