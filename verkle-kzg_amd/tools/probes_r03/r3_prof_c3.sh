#!/bin/bash
# C3 table traffic per geometry: FETCH_SIZE / WRITE_SIZE of k_fb_commit_cm for one table each
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-prof_c3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for G in 18:14 20 16; do
  T=$(echo $G | tr : _)
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch_$T -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/commit_breakdown.py $G > $O/fetch_$T.txt 2>&1 || exit 1
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write_$T -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/commit_breakdown.py $G > $O/write_$T.txt 2>&1 || exit 1
done
