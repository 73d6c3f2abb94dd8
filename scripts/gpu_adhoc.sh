set -eu
R=$(pwd)
O=$R/gpurun_out/r06_partM; mkdir -p $O
bash scripts/ab_probe.sh $O VKZG_MSM_M "16 24 32" 2 200 python -u verkle-kzg_amd/tools/split_probe.py 8
