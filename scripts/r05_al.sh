#!/bin/bash
# round 5 step AL/AM: the verkle sparse levels normalised through normalize_rows_items (polled block
# products, items and mirror placement fused, next level's lists built under the kernels) and the
# forward products taken as the flags arrive: verkle / msm / group / threads GPU tests, then
# verkle_ab.py against the library one change earlier (3 alternating rounds), then a kernel + copy
# trace of the new library
set -u
O=gpurun_out/r05_al
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_msm.py tests/test_gpu_group.py tests/test_gpu_threads.py tests/test_gpu_scheme.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
CUR=$(pwd)/verkle-kzg_amd/lib/libvkzg.so
PREV=$(pwd)/verkle-kzg_amd/lib_ab/libvkzg_prev.so
export VKZG_AB_FB_C=16
bash scripts/ab_probe.sh $O VKZG_LIB "$CUR $PREV" 3 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 || exit $?
for f in $O/VKZG_LIB_*; do echo "$f: $(tail -1 $f | cut -c1-200)"; done
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/tr -o vk -- python3 -u $R/verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $R/$O/trace_run.txt 2>&1; rc=$?
echo "trace rc=$rc"; grep full_ms $R/$O/trace_run.txt
exit $rc
