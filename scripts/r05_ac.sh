#!/bin/bash
# round 5 step AC: verkle laps on the final library (16-bit SRS windows), full + update
set -u
O=gpurun_out/r05_ac
mkdir -p $O
export TMPDIR=/tmp
VKZG_AB_FB_C=16 VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $O/laps.txt 2>&1 || exit $?
VKZG_AB_FB_C=16 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 6 > $O/ab.txt 2>&1 || exit $?
tail -1 $O/ab.txt
