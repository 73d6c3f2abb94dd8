#!/bin/bash
# rocprofv3 kernel trace of the 2^20 BLS12-381 MSM probe under each VKZG_ACC_MERGE value
# (straddle merge inside the accumulate on / off): per-kernel durations of the accumulate and the
# fix-up from the profiler, not the HIP-event timers.  usage: bash scripts/prof_merge.sh OUT
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$(mkdir -p "$1" && cd "$1" && pwd)
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
    VKZG_ACC_MERGE=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/m$v" -o run --output-format csv \
        -- python3 "$R/verkle-kzg_amd/tools/msm_probe.py" bls12_381 20 > "$OUT/m$v.log" 2>&1
    echo "merge=$v done"
done
