#!/bin/bash
# round 5 step AP: the per-rank G = 8 slices with the fix-up as a lane per owner thread
# (k_msm_fixup_own, default) vs a quad per bucket (k_msm_fixup_walk_q: VKZG_FIXUP_OWN=0), 2 rounds
set -u
O=gpurun_out/r05_ap
mkdir -p $O
export TMPDIR=/tmp
bash scripts/ab_probe.sh $O VKZG_FIXUP_OWN "1 0" 2 200 python -u verkle-kzg_amd/tools/split_probe.py 8 || exit $?
for f in $O/VKZG_FIXUP_OWN_*; do echo "== $f"; grep "G=8" $f | sed -e "s/{'glv_split.*msm_accumulate/{.. acc/" | cut -c1-200; done
