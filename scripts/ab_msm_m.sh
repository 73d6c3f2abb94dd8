# A/B of the accumulate's entries per thread (VKZG_MSM_M) for small per-window MSMs
set -o pipefail
O=${1:-gpurun_out/h28}
mkdir -p $O
run() { echo "== $*" >> $O/ab.txt; timeout -k 10 120 "$@" >> $O/ab.txt 2>&1 || exit $?; }
for n in 10 12 14 15 16; do for m in 4 8 16; do run env VKZG_MSM_M=$m python -u verkle-kzg_amd/tools/msm_probe.py bn254 $n; done; done
