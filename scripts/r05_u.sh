#!/bin/bash
# round 5 step U: verkle commitment without the dense level's stream wait and the root read-back
# (the root's point from the host-result level; one sync at the end): verkle / group tests, then
# alternating verkle_ab.py against the library one change earlier (lib_ab/libvkzg_verkle_prev.so)
set -u
O=gpurun_out/r05_u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_group.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
CUR=$(pwd)/verkle-kzg_amd/lib/libvkzg.so
PREV=$(pwd)/verkle-kzg_amd/lib_ab/libvkzg_verkle_prev.so
bash scripts/ab_probe.sh $O VKZG_LIB "$CUR $PREV" 3 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 || exit $?
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/laps.txt 2>&1 || exit $?
for f in $O/VKZG_LIB_*; do echo "$f: $(tail -1 $f)"; done
grep -E "root|final sync|dense" $O/laps.txt | tail -6
