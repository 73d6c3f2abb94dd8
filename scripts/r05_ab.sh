#!/bin/bash
# round 5 step AB: the IPA prover's rows made in the round kernel (IpaRows: coefficient rows folded
# on the device, the host keeps a, b and the q terms) and cached Python limbs: every -m gpu test,
# then alternating ipa_abi_probe.py / mp_probe.py with VKZG_IPA_DEV_ROWS 1 / 0
set -u
O=gpurun_out/r05_ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_probe.sh $O VKZG_IPA_DEV_ROWS "1 0" 3 200 python -u verkle-kzg_amd/tools/ipa_abi_probe.py || exit $?
bash scripts/ab_probe.sh $O/mp VKZG_IPA_DEV_ROWS "1 0" 2 200 python -u verkle-kzg_amd/tools/mp_probe.py 16 || exit $?
for f in $O/VKZG_IPA_DEV_ROWS_*; do echo "$f: $(tail -1 $f)"; done
for f in $O/mp/VKZG_IPA_DEV_ROWS_*; do echo "$f: $(grep -E 'finish' $f | tail -2 | tr '\n' ' ')"; done
