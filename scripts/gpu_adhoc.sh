set -eu
R=$(pwd)
O=$R/gpurun_out/r06_o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_verkle.py tests/test_gpu_verkle32.py tests/test_gpu_msm.py tests/test_gpu_scheme.py tests/test_gpu_group.py tests/test_gpu_comm.py > $O/tests.txt 2>&1
echo tests-ok; tail -2 $O/tests.txt
CUR=$R/verkle-kzg_amd/lib/libvkzg.so
PREV=$R/verkle-kzg_amd/lib_ab/libvkzg_r05.so
export VKZG_AB_FB_C=16
bash scripts/ab_probe.sh $O/verkle VKZG_LIB "$CUR $PREV" 3 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6
for f in $O/verkle/VKZG_LIB_*; do echo "$f: $(tail -1 $f | cut -c1-250)"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o vk -- python3 -u $R/verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/trace_run.txt 2>&1
echo trace-done
