#!/bin/bash
# round-3 probe batch 14: IPA prove round timeline (kernel + memory-copy trace)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3t}
mkdir -p $O
cd $R
timeout -k 10 120 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_probe.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/ipa_probe.py > $O/trace.txt 2>&1 || exit 1
