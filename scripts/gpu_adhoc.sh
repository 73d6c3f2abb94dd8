set -eu
R=$(pwd)
O=$R/gpurun_out/r06_h; mkdir -p $O
timeout -k 10 120 $R/verkle-kzg_amd/tools/affine_probe 32 3 > $O/affine_probe.txt 2>&1
echo probe-ok; cat $O/affine_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/pmc -o run -- $R/verkle-kzg_amd/tools/affine_probe 32 1 > $O/affine_probe_pmc_run.txt 2>&1
echo pmc-ok
find $O/pmc -name "*.csv" | head
