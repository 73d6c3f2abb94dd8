#!/bin/bash
# round 5 step AN: the verkle normalisation's block products scanned on the device (the last block
# to arrive; the host inverts one total): verkle / msm / group / threads / scheme GPU tests, then
# VKZG_NORM_DEVSCAN 1 / 0 alternating on verkle_ab.py (3 rounds), then a kernel + copy trace
set -u
O=gpurun_out/r05_an
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_msm.py tests/test_gpu_group.py tests/test_gpu_threads.py tests/test_gpu_scheme.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
export VKZG_AB_FB_C=16
bash scripts/ab_probe.sh $O VKZG_NORM_DEVSCAN "1 0" 3 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 || exit $?
for f in $O/VKZG_NORM_DEVSCAN_*; do echo "$f: $(tail -1 $f | cut -c1-200)"; done
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/tr -o vk -- python3 -u $R/verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $R/$O/trace_run.txt 2>&1; rc=$?
echo "trace rc=$rc"; grep full_ms $R/$O/trace_run.txt
exit $rc
