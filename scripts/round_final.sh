#!/bin/bash
# Round-end rehearsal on one MI355X: every -m gpu test, smoke(), the default bench line (with the
# CPU baselines), then the rocprofv3 kernel-trace + PMC passes of scripts/bench_profile.sh.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo tests-done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo smoke-done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
echo bench-done
[ "${2:-}" = "noprof" ] || bash $R/scripts/bench_profile.sh $TAG
