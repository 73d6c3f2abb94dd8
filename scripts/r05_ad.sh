#!/bin/bash
# round 5 step AD: the verkle levels' latency-path threshold at 16-bit SRS windows
# (VKZG_SPARSE_SMALL_MAX 2^18 (default) / 2^20 / 2^21 (non-zero, window) pairs), 2 alternating rounds
set -u
O=gpurun_out/r05_ad
mkdir -p $O
export TMPDIR=/tmp
export VKZG_AB_FB_C=16
bash scripts/ab_probe.sh $O VKZG_SPARSE_SMALL_MAX "262144 1048576 2097152" 2 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 || exit $?
for f in $O/VKZG_SPARSE_SMALL_MAX_*; do echo "$f: $(tail -1 $f | grep -o 'full_median_2+=[0-9.]* update_median_2+=[0-9.]*')"; done
