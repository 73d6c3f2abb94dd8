#!/bin/bash
# round-3 probe batch 4: dispatch gaps (stream vs graph), per-thread contexts, IPA bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3j}
mkdir -p $O
cd $R
timeout -k 10 60 verkle-kzg_amd/tools/gapprobe > $O/gapprobe.json 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_threads.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-secondary --no-verkle --no-cpu-baseline --no-variable-base --no-kzg --no-mp > $O/bench.json 2> $O/bench.err || exit 1
