#!/bin/bash
# A/B probe of one engine knob (an environment variable the library reads, e.g. VKZG_SORT_CSTAGE,
# VKZG_TAIL_MARGINAL, VKZG_RADIX_HIST) on the GPU box: the probe command runs under each value in
# turn, ROUNDS times alternating (box clocks drift; alternation keeps the comparison fair), one
# output file per (value, round), every step under its own time limit; stops at the first step
# that fails.
#   bash scripts/ab_probe.sh OUT VAR "v1 v2 ..." ROUNDS SECONDS command args...
# e.g. bash scripts/ab_probe.sh gpurun_out/ab_cstage VKZG_SORT_CSTAGE "1 0" 2 120 \
#          python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20
# Round 3's 23 batch scripts (verkle-kzg_amd/tools/probes_r03/README.md lists which knob and
# command each ran) are instances of this one.
set -u
OUT=$1; VAR=$2; VALUES=$3; ROUNDS=$4; SECS=$5; shift 5
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
    for v in $VALUES; do
        f="$OUT/${VAR}_$(basename "$v")_r$r.txt"  # a path value (VKZG_LIB=...) by its file name
        env "$VAR=$v" timeout -k 10 "$SECS" "$@" > "$f" 2>&1
        rc=$?
        echo "$VAR=$v round $r rc=$rc -> $f"
        [ $rc -eq 0 ] || exit $rc
    done
done
