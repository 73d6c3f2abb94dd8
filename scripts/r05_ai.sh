#!/bin/bash
# round 5 step AI: sort chunk (scalars per coarse block) 4096 (default) / 2048 / 1024 on the 2^20
# radix MSM: msm_probe.py kernel times, 2 alternating rounds (no code change: VKZG_SORT_CHUNK)
set -u
O=gpurun_out/r05_ai
mkdir -p $O
export TMPDIR=/tmp
bash scripts/ab_probe.sh $O VKZG_SORT_CHUNK "4096 2048 1024" 2 150 python -u verkle-kzg_amd/tools/msm_probe.py bls12_381 20 || exit $?
for f in $O/VKZG_SORT_CHUNK_*; do echo "$f: $(grep wall $f | cut -c1-60) | $(grep -E 'glv_split|sort_hist|scan|sort_coarse|sort_fine' $f | tr -s ' ' | tr '\n' ' ')"; done
