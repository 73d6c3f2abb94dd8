set -eu
R=$(pwd)
O=$R/gpurun_out/r06_fencefree; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_verkle.py tests/test_gpu_verkle32.py tests/test_gpu_msm.py::test_batch_commit_sparse_fused_equals_launches tests/test_gpu_msm.py::test_batch_commit_sparse -m gpu > $O/tests.txt 2>&1
echo tests-done; tail -2 $O/tests.txt
cd /tmp && export TMPDIR=/tmp
VKZG_AB_FB_C=16 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 -u $R/verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/trace_run.txt 2>&1
echo trace-done
cd $R
VKZG_AB_FB_C=16 bash scripts/ab_probe.sh $O/ab_fused VKZG_SPARSE_FUSED "1 0" 3 180 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 8
VKZG_AB_FB_C=16 bash scripts/ab_probe.sh $O/ab_tags VKZG_NORM_TAGS "1 0" 3 180 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 8
