# round 5 step A: new group tests, untimed MSM timeline (real inter-kernel gaps), bench
set -u
O=gpurun_out/r05_a
mkdir -p $O
R=$(pwd)
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_group.py tests/test_abi.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/msm_once.py bls12_381 20 10 > $R/$O/trace.log 2>&1 || exit $?
cd $R
python verkle-kzg_amd/tools/gap_report.py $O/trace/run_kernel_trace.csv k_glv_radix > $O/gaps.txt 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
