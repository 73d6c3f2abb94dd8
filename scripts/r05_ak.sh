#!/bin/bash
# round 5 step AK: kernel + copy trace of the verkle full commitment (65,536 keys, 16-bit SRS
# windows, 3 reps of verkle_ab.py) to locate the GPU idle gaps the host leaves
set -u
O=gpurun_out/r05_ak
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
VKZG_AB_FB_C=16 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o vk -- python3 -u $GRAFT_REPO_ROOT/verkle-kzg_amd/tools/verkle_ab.py 65536 3 > $GRAFT_REPO_ROOT/$O/run.txt 2>&1; rc=$?
echo "rc=$rc"; tail -3 $GRAFT_REPO_ROOT/$O/run.txt
find $GRAFT_REPO_ROOT/$O/tr -name "*.csv" | head
exit $rc
