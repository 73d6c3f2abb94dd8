# round 5 step F: verkle latency path (wave per 64 pairs) + delta rows + fused normalisation;
# verkle tests, node diagnostic, A/B (small path on/off, delta on/off), update trace
set -u
O=gpurun_out/r05_f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_group.py tests/test_gpu_msm.py -k "verkle or sparse" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_nodes.py > $O/nodes.txt 2>&1 || exit $?
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 > $O/ab.txt 2>&1 || exit $?
VKZG_VERKLE_DELTA=0 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 >> $O/ab.txt 2>&1 || exit $?
VKZG_SPARSE_SMALL_MAX=0 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 >> $O/ab.txt 2>&1 || exit $?
VKZG_SPARSE_SMALL_MAX=2000000 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 >> $O/ab.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/vtrace -o vt -- python3 -u verkle-kzg_amd/tools/verkle_ab.py 65536 2 > $O/vtrace.log 2>&1 || exit $?
