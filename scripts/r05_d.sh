# round 5 step D: the whole GPU suite after the 128-B fixed-base entries + device verkle levels; verkle A/B
set -u
O=gpurun_out/r05_d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_nodes.py > $O/nodes.txt 2>&1 || exit $?
for v in 1 1; do
  VKZG_VERKLE_DEV=$v timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 >> $O/ab.txt 2>&1 || exit $?
done
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/laps_dev.txt 2>&1 || exit $?
