set -eu
R=$(pwd)
O=$R/gpurun_out/r06_n; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
VKZG_AB_FB_C=16 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o vk -- python3 -u $R/verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/trace_run.txt 2>&1
echo trace-done; tail -1 $O/trace_run.txt | cut -c1-200
find $O/tr -name "*.csv" | head
