# round 5 step H: IPA strided compaction, verkle delta plan on per-node arrays + reused ext parts:
# tests, verkle A/B + laps, IPA A/B (compact on / off, alternating)
set -u
O=gpurun_out/r05_h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verkle.py tests/test_gpu_group.py tests/test_gpu_msm.py tests/test_gpu_scheme.py tests/test_gpu_multiproof_256.py -k "verkle or sparse or ipa or commit or multiproof" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_nodes.py > $O/nodes.txt 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 >> $O/ab.txt 2>&1 || exit $?
  timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_c1_$k.txt 2>&1 || exit $?
  VKZG_IPA_COMPACT=0 timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_c0_$k.txt 2>&1 || exit $?
done
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/laps.txt 2>&1 || exit $?
