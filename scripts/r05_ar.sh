#!/bin/bash
# round 5 step AR: sparse commits whose rows are single chunks skip k_sparse_combine (the chunk
# sums are the rows): verkle / msm GPU tests, then verkle_ab.py against the library one change
# earlier (3 alternating rounds)
set -u
O=gpurun_out/r05_ar
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_msm.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
CUR=$(pwd)/verkle-kzg_amd/lib/libvkzg.so
PREV=$(pwd)/verkle-kzg_amd/lib_ab/libvkzg_prev.so
export VKZG_AB_FB_C=16
bash scripts/ab_probe.sh $O VKZG_LIB "$CUR $PREV" 3 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 7 || exit $?
for f in $O/VKZG_LIB_*; do echo "$(basename $f): $(tail -1 $f | cut -c60-230)"; done
