# round 5 step C: verkle device path v2 (inline leaves, compact flags, mirror fixes) -- tests and A/B
set -u
O=gpurun_out/r05_c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_group.py tests/test_gpu_fullsize.py -k "verkle or commit_10k" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 1; do
  VKZG_VERKLE_DEV=$v timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 >> $O/ab.txt 2>&1 || exit $?
done
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/laps_dev.txt 2>&1 || exit $?
