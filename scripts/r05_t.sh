#!/bin/bash
# round 5 step T: latency-path commits adding each block partial as its flag arrives
# (VKZG_SMALL_INCR 1 / 0): every -m gpu test, then alternating IPA / multiproof probes
set -u
O=gpurun_out/r05_t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_probe.sh $O VKZG_SMALL_INCR "1 0" 3 150 python -u verkle-kzg_amd/tools/ipa_probe.py || exit $?
bash scripts/ab_probe.sh $O/mp VKZG_SMALL_INCR "1 0" 2 200 python -u verkle-kzg_amd/tools/mp_probe.py 16 || exit $?
for f in $O/VKZG_SMALL_INCR_*; do echo "$f: $(grep -E '^prove' $f)"; done
for f in $O/mp/VKZG_SMALL_INCR_*; do echo "$f: $(grep -E 'finish' $f | head -3 | tr '\n' ' ')"; done
