# round 5 step J: verkle host stage (no false sharing in the row parts, branch-light stem items):
# verkle tests, host-stage probe, verkle A/B + laps
set -u
O=gpurun_out/r05_j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_group.py -k "verkle" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_host_probe.py 65536 15 > $O/host_probe.txt 2>&1 || exit $?
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_nodes.py > $O/nodes.txt 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 >> $O/ab.txt 2>&1 || exit $?
done
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/laps.txt 2>&1 || exit $?
