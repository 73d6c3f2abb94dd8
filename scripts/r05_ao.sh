#!/bin/bash
# round 5 step AO: width-4 row pointers kept between calls (verkle GPU tests + verkle_ab.py), and the
# one-card per-rank MSM slices timed without per-kernel events (split_probe.py: wall time first,
# then the instrumented loop for the kernel breakdown)
set -u
O=gpurun_out/r05_ao
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u verkle-kzg_amd/tools/split_probe.py 1,2,8 > $O/split_probe.txt 2>&1; rc=$?
echo "split rc=$rc"; cut -c1-110 $O/split_probe.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verkle.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
VKZG_AB_FB_C=16 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 7 > $O/verkle_ab.txt 2>&1; rc=$?
tail -1 $O/verkle_ab.txt | cut -c1-220
exit $rc
