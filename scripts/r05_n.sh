# round 5 step N: verkle normalisation with polled flags (zero copies): verkle + group tests, A/B
set -u
O=gpurun_out/r05_n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_group.py -k "verkle" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_nodes.py > $O/nodes.txt 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 >> $O/ab.txt 2>&1 || exit $?
done
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_bench_seq.py 1 6 > $O/seq.txt 2>&1 || exit $?
