#!/bin/bash
# round 5 step V: multiproof finish with D / E committed from device scalars (no g / h read-back,
# no stream waits; h - g copied into page-locked memory ahead of E): multiproof / scheme tests,
# then alternating mp_probe.py against the library one change earlier (lib_ab/libvkzg_prev.so)
set -u
O=gpurun_out/r05_v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multiproof_256.py tests/test_gpu_scheme.py tests/test_gpu_group.py tests/test_gpu_comm.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
CUR=$(pwd)/verkle-kzg_amd/lib/libvkzg.so
PREV=$(pwd)/verkle-kzg_amd/lib_ab/libvkzg_prev.so
bash scripts/ab_probe.sh $O VKZG_LIB "$CUR $PREV" 3 200 python -u verkle-kzg_amd/tools/mp_probe.py 16 || exit $?
for f in $O/VKZG_LIB_*; do echo "$f: $(grep -E 'finish' $f | tail -2 | tr '\n' ' ')"; done
