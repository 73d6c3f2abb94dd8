set -eu
R=$(pwd)
O=$R/gpurun_out/r06_lead4t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 20 0 18; do
VKZG_VERKLE_LEAD_C=$v VKZG_AB_FB_C=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o run -- python3 -u $R/verkle-kzg_amd/tools/verkle_ab.py 65536 4 > $O/run_$v.txt 2>&1
done
echo done
