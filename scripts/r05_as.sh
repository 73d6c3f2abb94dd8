#!/bin/bash
# round 5 step AS: the MSM fix-up as the owner walk (default) vs guarded pointer-jumping rounds
# (VKZG_MSM_FIXUP=1), 2 alternating rounds of msm_probe.py bls12_381 20
set -u
O=gpurun_out/r05_as
mkdir -p $O
export TMPDIR=/tmp
bash scripts/ab_probe.sh $O VKZG_MSM_FIXUP "0 1" 2 200 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 || exit $?
for f in $O/VKZG_MSM_FIXUP_*; do echo "$(basename $f): $(grep -E 'wall|msm_fixup|msm_segsum' $f | tr -s ' ' | tr '\n' ' ' | cut -c1-220)"; done
