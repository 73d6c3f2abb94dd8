#!/bin/bash
# Round-5 rehearsal on one MI355X, in the order that ties the bench line to its counters: every
# -m gpu test, smoke(), the rocprofv3 kernel trace + PMC passes of the bench (scripts/bench_profile.sh),
# their summary installed as profiles/r05/pmc_summary.json (so the bench line reads counters taken on
# this library), then the default bench line with the CPU baselines.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05_final}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo tests-done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo smoke-done
bash $R/scripts/bench_profile.sh $TAG
cp $R/gpurun_out/prof_$TAG/summary.json $R/profiles/r05/pmc_summary.json
mkdir -p $O/profiles_r05 && cp $R/profiles/r05/pmc_summary.json $O/profiles_r05/
cd $R
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
echo bench-done
# the N > 1 flow end to end (two ranks on this one card, gloo + host-callback exchange)
timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline > $O/rehearse_2rank.json 2> $O/rehearse_2rank.err
echo rehearse-done
# one-card per-rank slices of the 2^20 MSM (point ranges / window parts at G = 2 and 8)
timeout -k 10 300 python -u verkle-kzg_amd/tools/split_probe.py 1,2,8 > $O/split_probe.txt 2>&1
echo split-done
