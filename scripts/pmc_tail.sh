#!/bin/bash
# Counter list of the box, then SQ issue / stall counters of the 2^20 BLS12-381 MSM probe's kernels
# (accumulate vs the latency-bound fix-up and reduction): one PMC pass, kernel trace on.
#   bash scripts/pmc_tail.sh OUT
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$(mkdir -p "$1" && cd "$1" && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
echo list-done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES \
    -d "$OUT/sq" -o run --output-format csv -- python3 "$R/verkle-kzg_amd/tools/msm_probe.py" bls12_381 20 > "$OUT/sq.log" 2>&1
echo sq-done
