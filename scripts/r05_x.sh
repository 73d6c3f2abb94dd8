#!/bin/bash
# round 5 step X: lazily built fixed-base tables sized by a 20 GB budget (the 257-point IPA CRS at
# c = 16): every -m gpu test (time / memory), smoke; then the verkle commitment at window bits
# 8 / 12 / 16 for the KZG(256) SRS table (VKZG_AB_FB_C in verkle_ab.py)
set -u
O=gpurun_out/r05_x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --durations=15 > $O/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -22 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_probe.sh $O VKZG_AB_FB_C "8 12 16" 2 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 || exit $?
for f in $O/VKZG_AB_FB_C_*; do echo "$f: $(tail -1 $f | grep -o 'full_median_2+=[0-9.]* update_median_2+=[0-9.]*')"; done
