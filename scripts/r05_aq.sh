#!/bin/bash
# round 5 step AQ: k_glv_radix_hist with its per-lane scalar loop unrolled (no scratch-memory
# indexing) vs the library one change earlier: msm GPU tests, then msm_probe.py 3 alternating rounds
set -u
O=gpurun_out/r05_aq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_fullsize.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
CUR=$(pwd)/verkle-kzg_amd/lib/libvkzg.so
PREV=$(pwd)/verkle-kzg_amd/lib_ab/libvkzg_prev.so
bash scripts/ab_probe.sh $O VKZG_LIB "$CUR $PREV" 3 200 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 || exit $?
for f in $O/VKZG_LIB_*; do echo "== $f"; grep -v amdgpu.ids $f | tail -4 | cut -c1-260; done
