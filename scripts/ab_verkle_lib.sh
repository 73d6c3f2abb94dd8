# A/B of two library builds on the verkle full commitment (VKZG_LIB=<alt> vs the default), 3
# alternating rounds of tools/verkle_probe.py with the VKZG_VERBOSE laps
set -o pipefail
O=${1:-gpurun_out/verkle_ab}; ALT=${2:-verkle-kzg_amd/lib/libvkzg_ab.so}
mkdir -p $O
for r in 1 2 3; do
  echo "== round $r alt ($ALT)" >> $O/ab.txt
  timeout -k 10 120 env VKZG_LIB=$ALT VKZG_VERBOSE=1 python -u verkle-kzg_amd/tools/verkle_probe.py >> $O/ab.txt 2>&1 || exit $?
  echo "== round $r default" >> $O/ab.txt
  timeout -k 10 120 env VKZG_VERBOSE=1 python -u verkle-kzg_amd/tools/verkle_probe.py >> $O/ab.txt 2>&1 || exit $?
done
