#!/bin/bash
# round-3 probe batch 2: batched-MSM / fused-KZG tests, kernel timeline gaps of one MSM and of an
# 8-rank window slice, KZG + multiproof bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3h}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "many or kzg" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-secondary --no-verkle --no-ipa --no-cpu-baseline --no-variable-base > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/msm_probe.py bls12_381 20 > $O/trace_probe.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace8 -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/slice_trace.py > $O/trace8_probe.txt 2>&1 || exit 1
