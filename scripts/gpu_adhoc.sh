set -eu
R=$(pwd)
O=$R/gpurun_out/r06_m; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_verkle.py tests/test_gpu_verkle32.py tests/test_gpu_group.py tests/test_gpu_comm.py > $O/tests.txt 2>&1
echo tests-ok; tail -2 $O/tests.txt
export VKZG_AB_FB_C=16
bash scripts/ab_probe.sh $O/pieces VKZG_VERKLE_EXT_PIECES "4 1 2" 3 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6
for f in $O/pieces/VKZG_*; do echo "$f: $(tail -1 $f | cut -c1-250)"; done
