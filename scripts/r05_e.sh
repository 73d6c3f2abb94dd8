# round 5 step E: whole GPU suite (sort preloads, pinned verkle merge, identity chunks, one-block
# mirror), MSM timeline, verkle A/B + update trace, the group probe on one card
set -u
O=gpurun_out/r05_e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_nodes.py > $O/nodes.txt 2>&1 || exit $?
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 > $O/ab.txt 2>&1 || exit $?
VKZG_VERKLE_DELTA=0 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 5 >> $O/ab.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/vtrace -o vt -- python3 -u verkle-kzg_amd/tools/verkle_ab.py 65536 2 > $O/vtrace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/msm -o msm -- python3 -u verkle-kzg_amd/tools/msm_once.py > $O/msm.log 2>&1 || exit $?
timeout -k 10 300 python -u verkle-kzg_amd/tools/group_probe.py > $O/group.txt 2>&1 || exit $?
