#!/bin/bash
# round 5 step S: divstep host inversion + polled MSM tail: every -m gpu test, then the bench
# lines without CPU baselines / configs[2] (headline, IPA, multiproof, KZG, verkle)
set -u
O=gpurun_out/r05_s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-secondary > $O/bench.json 2> $O/bench.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r05_s/bench.json"))
print("headline", d["ms_per_step"], d.get("ms_per_step_median"))
for k in ("ipa", "multiproof", "verkle", "kzg"):
    v = d.get(k)
    if isinstance(v, dict):
        print(k, {kk: vv for kk, vv in v.items() if isinstance(vv, (int, float))})
PY
