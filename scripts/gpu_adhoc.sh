set -eu
R=$(pwd)
O=$R/gpurun_out/r06_l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_verkle.py tests/test_gpu_verkle32.py > $O/tests.txt 2>&1
echo tests-ok; tail -2 $O/tests.txt
CUR=$R/verkle-kzg_amd/lib/libvkzg.so
PREV=$R/verkle-kzg_amd/lib_ab/libvkzg_r05.so
export VKZG_AB_FB_C=16
bash scripts/ab_probe.sh $O/verkle VKZG_LIB "$CUR $PREV" 3 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6
for f in $O/verkle/VKZG_LIB_*; do echo "$f: $(tail -1 $f | cut -c1-250)"; done
bash scripts/ab_probe.sh $O/group VKZG_LIB "$CUR $PREV" 2 300 python -u verkle-kzg_amd/tools/group_mp_probe.py 14 4 3
for f in $O/group/VKZG_LIB_*; do echo "$f: $(tail -1 $f)"; done
WPE3=$R/verkle-kzg_amd/lib_ab/libvkzg_wpe3.so
bash scripts/ab_probe.sh $O/wpe3 VKZG_LIB "$CUR $WPE3" 3 120 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20
for f in $O/wpe3/VKZG_LIB_*; do echo "$f: $(grep -E 'wall|msm_accumulate' $f | tr '\n' ' ' | cut -c1-250)"; done
