#!/bin/bash
# round-3 probe batch 16: verkle full commitment, new host staging vs the previous library (A/B)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3w}
mkdir -p $O
cd $R
V=verkle-kzg_amd/tools/verkle_probe.py
for i in 1 2; do
REPS=8 timeout -k 10 200 python -u $V > $O/new$i.txt 2>&1 || exit 1
VKZG_LIB=$R/verkle-kzg_amd/lib/libvkzg_old.so REPS=8 timeout -k 10 200 python -u $V > $O/old$i.txt 2>&1 || exit 1
done
