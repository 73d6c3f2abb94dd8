#!/bin/bash
# round 5 step AA: IPA host micro-steps (cached domain generator, zero-skipping inner products,
# round 0 rows without multiplies): scheme / multiproof tests, then alternating ipa_abi_probe.py
# against the library one change earlier (lib_ab/libvkzg_prev.so)
set -u
O=gpurun_out/r05_aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scheme.py tests/test_gpu_multiproof_256.py tests/test_gpu_verkle.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
CUR=$(pwd)/verkle-kzg_amd/lib/libvkzg.so
PREV=$(pwd)/verkle-kzg_amd/lib_ab/libvkzg_prev.so
bash scripts/ab_probe.sh $O VKZG_LIB "$CUR $PREV" 3 200 python -u verkle-kzg_amd/tools/ipa_abi_probe.py || exit $?
for f in $O/VKZG_LIB_*; do echo "$f: $(tail -1 $f)"; done
