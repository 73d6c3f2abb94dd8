# round 5 step O: latency-path block size A/B (VKZG_SMALL_NT 256 / 128 / 64): IPA probe with host laps
set -u
O=gpurun_out/r05_o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scheme.py -k "ipa" > $O/tests.txt 2>&1 || exit $?
for nt in 256 128 64; do
  VKZG_SMALL_NT=$nt timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scheme.py -k "ipa" >> $O/tests_nt.txt 2>&1 || exit $?
  VKZG_SMALL_NT=$nt timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_nt$nt.txt 2>&1 || exit $?
  VKZG_SMALL_NT=$nt VKZG_HOST_TIMING=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_nt${nt}_laps.txt 2>&1 || exit $?
done
