# round 5 step G: verkle v2 (NT per level, lists built during the wait) + IPA compacted rounds:
# verkle + IPA + commit tests, verkle A/B, update trace, IPA probe with host laps
set -u
O=gpurun_out/r05_g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_group.py tests/test_gpu_msm.py tests/test_gpu_scheme.py -k "verkle or sparse or ipa or commit" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_nodes.py > $O/nodes.txt 2>&1 || exit $?
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 > $O/ab.txt 2>&1 || exit $?
VKZG_SPARSE_SMALL_MAX=2000000 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 >> $O/ab.txt 2>&1 || exit $?
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 >> $O/ab.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/vtrace -o vt -- python3 -u verkle-kzg_amd/tools/verkle_ab.py 65536 2 > $O/vtrace.log 2>&1 || exit $?
VKZG_HOST_TIMING=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa.txt 2>&1 || exit $?
VKZG_IPA_COMPACT=0 timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_nocompact.txt 2>&1 || exit $?
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/laps.txt 2>&1 || exit $?
