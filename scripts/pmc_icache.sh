#!/bin/bash
# Instruction-cache counters of the 2^20 BLS12-381 MSM probe's kernels (are the latency-bound tail
# kernels -- one straight-line EC add per wave -- instruction-fetch bound?): one PMC pass.
#   bash scripts/pmc_icache.sh OUT
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$(mkdir -p "$1" && cd "$1" && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_WAVE_CYCLES \
    -d "$OUT/ic" -o run --output-format csv -- python3 "$R/verkle-kzg_amd/tools/msm_probe.py" bls12_381 20 > "$OUT/ic.log" 2>&1
echo icache-done
