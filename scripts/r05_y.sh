#!/bin/bash
# round 5 step Y: the headline step vs the number of untimed warm-up steps (3 / 20 / 100), 20 timed
# steps, 2 alternating rounds (headline only)
set -u
O=gpurun_out/r05_y
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for w in 3 20 100; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup $w --no-cpu-baseline --no-secondary --no-kzg --no-mp --no-verkle --no-ipa --no-variable-base > $O/w${w}_r$r.json 2> $O/w${w}_r$r.err || exit $?
    python3 -c "import json;d=json.load(open('$O/w${w}_r$r.json'));print('warmup $w round $r', round(d['ms_per_step'],4), round(d['ms_per_step_median'],4), round(d['ms_per_step_min'],4), round(d['ms_per_step_with_events'],4), round(d['kernel_ms']['msm_accumulate'],4), round(d['accumulate_clock_mhz']))"
  done
done
