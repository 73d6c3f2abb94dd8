# round 5 step B: verkle device path -- tests, A/B of the two paths, laps of the device path
set -u
O=gpurun_out/r05_b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_group.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 0 1 0; do
  VKZG_VERKLE_DEV=$v timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 >> $O/ab.txt 2>&1 || exit $?
done
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/laps_dev.txt 2>&1 || exit $?
for lib in libvkzg.so libvkzg_pad128.so libvkzg.so libvkzg_pad128.so; do
  VKZG_LIB=$(pwd)/verkle-kzg_amd/lib/$lib timeout -k 10 300 python -u verkle-kzg_amd/tools/commit_ab.py 5 16:0 17:0 18:14 >> $O/commit_ab.txt 2>&1 || exit $?
done
