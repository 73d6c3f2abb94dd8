#!/bin/bash
# rocprofv3 recipe used for profiles/ (kernel trace + stats, then HBM PMC passes, then summary).
# usage: bash scripts/bench_profile.sh <tag> [bench args...]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_trace.json
echo trace-done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_fetch.json
echo fetch-done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_write.json
echo write-done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES -d $OUT/valu -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_valu.json
echo valu-done
python3 $R/verkle-kzg_amd/tools/prof_summary.py $OUT $OUT/summary.json
echo profile-done
