# round 5 step M: latency-path completion by polled flags (no stream wait): the latency-path users'
# tests, IPA / multiproof / verkle A/B (VKZG_SMALL_POLL 1 / 0, alternating)
set -u
O=gpurun_out/r05_m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scheme.py tests/test_gpu_multiproof_256.py tests/test_gpu_verkle.py tests/test_gpu_msm.py -k "ipa or multiproof or kzg or verkle or commit or batch" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_p1_$k.txt 2>&1 || exit $?
  VKZG_SMALL_POLL=0 timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_p0_$k.txt 2>&1 || exit $?
  timeout -k 10 200 python -u verkle-kzg_amd/tools/mp_probe.py 16 > $O/mp_p1_$k.txt 2>&1 || exit $?
  VKZG_SMALL_POLL=0 timeout -k 10 200 python -u verkle-kzg_amd/tools/mp_probe.py 16 > $O/mp_p0_$k.txt 2>&1 || exit $?
done
timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 > $O/verkle_p1.txt 2>&1 || exit $?
VKZG_SMALL_POLL=0 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 > $O/verkle_p0.txt 2>&1 || exit $?
