#!/bin/bash
# round-3 probe batch 3: mixed-window fixed-base tables (C3 from a <= 60 GB table)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3i}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py -k "mixed or batch_commit or sparse" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u verkle-kzg_amd/tools/commit_breakdown.py 18 18:14 19 > $O/commit.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fullsize.py -k "mixed" > $O/tests_full.txt 2>&1 || exit 1
