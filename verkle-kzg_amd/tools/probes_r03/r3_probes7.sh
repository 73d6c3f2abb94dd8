#!/bin/bash
# round-3 probe batch 7: kernel timeline of the one-call KZG commit + open (C4)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3m}
mkdir -p $O
cd $R
timeout -k 10 120 python -u verkle-kzg_amd/tools/kzg_trace.py fused > $O/kzg_wall.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/kzg_trace.py fused > $O/kzg_trace.txt 2>&1 || exit 1
