#!/bin/bash
# round-3 probe batch 8: sort geometry of the batched (K = 2) MSM inside the one-call KZG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3n}
mkdir -p $O
cd $R
K=verkle-kzg_amd/tools/kzg_trace.py
timeout -k 10 120 python -u $K fused > $O/default.txt 2>&1 || exit 1
VKZG_SORT_CHUNK=4096 timeout -k 10 120 python -u $K fused > $O/chunk4096.txt 2>&1 || exit 1
VKZG_SORT_CHUNK=2048 timeout -k 10 120 python -u $K fused > $O/chunk2048.txt 2>&1 || exit 1
VKZG_SORT_FB=6 timeout -k 10 120 python -u $K fused > $O/fb6.txt 2>&1 || exit 1
VKZG_SORT_FB=6 VKZG_SORT_CHUNK=4096 timeout -k 10 120 python -u $K fused > $O/fb6_chunk4096.txt 2>&1 || exit 1
timeout -k 10 120 python -u $K fused > $O/default2.txt 2>&1 || exit 1
