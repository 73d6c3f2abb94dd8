#!/bin/bash
# round 5 step AJ: the IPA prover's K rounds in one launch (k_ipa_rounds: resident blocks released
# round by round through coherent page-locked memory): scheme / multiproof / verkle / group /
# threads GPU tests, then VKZG_IPA_PERSIST 1 / 0 alternating on ipa_abi_probe.py and mp_probe.py
set -u
O=gpurun_out/r05_aj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scheme.py tests/test_gpu_multiproof_256.py tests/test_gpu_verkle.py tests/test_gpu_group.py tests/test_gpu_threads.py tests/test_gpu_comm.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_probe.sh $O VKZG_IPA_PERSIST "1 0" 3 200 python -u verkle-kzg_amd/tools/ipa_abi_probe.py || exit $?
bash scripts/ab_probe.sh $O/mp VKZG_IPA_PERSIST "1 0" 2 200 python -u verkle-kzg_amd/tools/mp_probe.py 16 || exit $?
for f in $O/VKZG_IPA_PERSIST_*; do echo "$f: $(tail -1 $f)"; done
for f in $O/mp/VKZG_IPA_PERSIST_*; do echo "$f: $(grep -E 'finish' $f | tail -2 | tr '\n' ' ' | cut -c1-160)"; done
