set -u
O=gpurun_out/r05_base
mkdir -p $O
timeout -k 10 120 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 > $O/probe.txt 2>&1 || exit $?
VKZG_HOST_TIMING=1 timeout -k 10 120 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 > $O/probe_ht.txt 2>&1 || exit $?
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/msm_probe.py bls12_381 20 > $R/$O/trace.log 2>&1 || exit $?
cd $R
f=$(ls $O/trace/*/run_kernel_trace.csv 2>/dev/null || ls $O/trace/run_kernel_trace.csv)
python verkle-kzg_amd/tools/gap_report.py $f k_glv_radix > $O/gaps.txt 2>&1
lscpu | head -20 > $O/lscpu.txt
