#!/bin/bash
# Round-end rehearsal on one MI355X, in the order that ties the bench line to its counters: every
# -m gpu test, smoke(), the rocprofv3 kernel trace + PMC passes of the bench (scripts/bench_profile.sh),
# their summary installed as profiles/<round>/pmc_summary.json (so the bench line reads counters taken
# on this library), the default bench line with the CPU baselines, the N > 1 flow on this one card
# (bench.py --gpus 2 --rehearse-one-gpu starts its two ranks itself), and the one-card split probe.
#   bash scripts/round_final.sh <round, e.g. r06> [tag] [noprof]
# (round 5's r05_final.sh and its ~45 one-shot job scripts were instances of this file and of
# scripts/ab_probe.sh; profiles/r05/INDEX.md keeps which command made which file)
set -e
RND=${1:-r06}
TAG=${2:-${RND}_final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O $R/profiles/$RND
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo tests-done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo smoke-done
if [ "${3:-}" != "noprof" ]; then
    bash $R/scripts/bench_profile.sh $TAG
    cp $R/gpurun_out/prof_$TAG/summary.json $R/profiles/$RND/pmc_summary.json
    mkdir -p $O/profiles_$RND && cp $R/profiles/$RND/pmc_summary.json $O/profiles_$RND/
fi
cd $R
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
echo bench-done
timeout -k 10 900 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline > $O/rehearse_2rank.json 2> $O/rehearse_2rank.err
echo rehearse-done
timeout -k 10 300 python -u verkle-kzg_amd/tools/split_probe.py 1,2,8 > $O/split_probe.txt 2>&1
echo split-done
