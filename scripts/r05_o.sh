# round 5 step O: latency-path block size (VKZG_SMALL_NT 256 / 128 / 64) x IPA host team
# (VKZG_IPA_TEAM 0 / 3 / 7 helpers): IPA tests per setting, probe times
set -u
O=gpurun_out/r05_o
mkdir -p $O
export TMPDIR=/tmp
for nt in 256 128 64; do
  for tm in 0 3 7; do
    VKZG_SMALL_NT=$nt VKZG_IPA_TEAM=$tm timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scheme.py -k "ipa" >> $O/tests.txt 2>&1 || exit $?
    echo "NT=$nt TEAM=$tm" >> $O/ipa.txt
    VKZG_SMALL_NT=$nt VKZG_IPA_TEAM=$tm timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py 2>&1 | grep -E "^(commit|prove|verify)" >> $O/ipa.txt || exit $?
  done
done
for nt in 256 64; do
  VKZG_SMALL_NT=$nt VKZG_IPA_TEAM=7 VKZG_HOST_TIMING=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_laps_nt$nt.txt 2>&1 || exit $?
done
