#!/bin/bash
# round-3 probe batch: window-slice scale probe (+ host phases), fixed-base commit window sweep,
# MSM host phases, sort geometry A/B (coarse bins x block size)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3g}
mkdir -p $O
cd $R/verkle-kzg_amd/tools
P="timeout -k 10 120 python -u msm_probe.py bls12_381 20"
VKZG_HOST_TIMING=1 $P > $O/probe.txt 2> $O/probe_host.txt || exit 1
for fb in 7 8; do for ch in 2048 4096 8192; do
  VKZG_SORT_FB=$fb VKZG_SORT_CHUNK=$ch $P > $O/sort_fb${fb}_ch${ch}.txt 2>&1 || exit 1
done; done
VKZG_HOST_TIMING=1 timeout -k 10 200 python -u scale_probe.py > $O/scale.txt 2> $O/scale_host.txt || exit 1
timeout -k 10 400 python -u commit_breakdown.py 16 17 18 19 20 > $O/commit.txt 2>&1 || exit 1
