#!/bin/bash
# same-box A/B of the radix-B shared-window MSM knobs (tools/msm_probe.py per setting)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep}
mkdir -p $O
cd $R/verkle-kzg_amd/tools
P="timeout -k 10 120 python -u msm_probe.py bls12_381 20"
if [ -x ./issueprobe ]; then timeout -k 10 60 ./issueprobe > $O/issueprobe.jsonl; fi
$P > $O/default.txt 2>&1
VKZG_SEGSUM_QUAD=0 $P > $O/segsum_lane.txt 2>&1
VKZG_FIXUP_QUAD=2 $P > $O/fixup_quad.txt 2>&1
VKZG_SORT_CHUNK=4096 $P > $O/chunk4096.txt 2>&1
VKZG_SORT_CHUNK=16384 $P > $O/chunk16384.txt 2>&1
VKZG_SORT_FB=6 $P > $O/fb6.txt 2>&1
VKZG_MSM_RADIX=1 $P > $O/c16.txt 2>&1
$P > $O/default2.txt 2>&1
