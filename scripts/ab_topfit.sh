set -o pipefail
O=gpurun_out/h26
mkdir -p $O
run() { echo "== $*" >> $O/ab.txt; timeout -k 10 120 "$@" >> $O/ab.txt 2>&1 || exit $?; }
for n in 12 14 15 16; do for tf in 0 1; do run env VKZG_MSM_TOPFIT=$tf python -u verkle-kzg_amd/tools/msm_probe.py bn254 $n; done; done
for q in 12 14 15; do for tf in 0 1; do run env VKZG_MSM_TOPFIT=$tf python -u verkle-kzg_amd/tools/mp_verify_probe.py $q 6; done; done
for n in 12 16; do for tf in 0 1; do run env VKZG_MSM_TOPFIT=$tf python -u verkle-kzg_amd/tools/msm_probe.py bandersnatch $n; done; done
