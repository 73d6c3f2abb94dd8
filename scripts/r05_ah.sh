#!/bin/bash
# round 5 step AH: the fine sort keeping a staged bin's entries in registers (read once) --
# MSM tests, then VKZG_SORT_FINE_REGS 1 / 0 alternating on msm_probe.py (kernel times)
set -u
O=gpurun_out/r05_ah
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_fullsize.py tests/test_gpu_kzg_device.py tests/test_gpu_group.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_probe.sh $O VKZG_SORT_FINE_REGS "1 0" 3 150 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 || exit $?
for f in $O/VKZG_SORT_FINE_REGS_*; do echo "$f: $(grep wall $f) $(grep sort_fine $f)"; done
