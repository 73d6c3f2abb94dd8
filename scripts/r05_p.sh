#!/bin/bash
# round 5 step P: the fix-up folded into the reduction's segment stage (k_msm_segr_fix_q): every
# -m gpu test, an alternating A/B of VKZG_TAIL_FUSE, and untimed kernel timelines of consecutive
# MSMs (the inter-call gap with direct completion on / off)
set -u
O=gpurun_out/r05_p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_probe.sh $O VKZG_TAIL_FUSE "1 0" 3 150 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 || exit $?
for f in $O/VKZG_TAIL_FUSE_*; do echo "$f: $(grep wall $f)"; grep -E "fixup|segsum" $f; done
for p in 1 0; do
  VKZG_TAIL_POLL=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_p$p -o run --output-format csv -- python3 verkle-kzg_amd/tools/msm_once.py bls12_381 20 10 > $O/trace_p$p.log 2>&1 || exit $?
  f=$(find $O/trace_p$p -name "run_kernel_trace.csv" | head -1)
  python verkle-kzg_amd/tools/timeline.py $f 40 > $O/timeline_p$p.txt 2>&1 || exit $?
done
