set -eu
R=$(pwd)
O=$R/gpurun_out/r06_normearly7; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_verkle.py tests/test_gpu_verkle32.py -m gpu > $O/tests.txt 2>&1
echo tests-done; tail -2 $O/tests.txt
VKZG_AB_FB_C=16 bash scripts/ab_probe.sh $O/ab VKZG_NORM_EARLY "1 0" 3 180 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 8
cd /tmp && export TMPDIR=/tmp
VKZG_AB_FB_C=16 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 -u $R/verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/trace_run.txt 2>&1
echo trace-done
