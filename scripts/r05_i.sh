# round 5 step I: configs[2] deployable table (c = 16 x 15 windows, 31.1 GB) timing + HBM PMC passes
set -u
O=gpurun_out/r05_i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u verkle-kzg_amd/tools/commit_ab.py 5 16:15 17:0 16:0 > $O/commit_ab.txt 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/verkle-kzg_amd/tools/commit_ab.py 3 16:15 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/fetch -o run -- python3 $GRAFT_REPO_ROOT/verkle-kzg_amd/tools/commit_ab.py 3 16:15 > $GRAFT_REPO_ROOT/$O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/write -o run -- python3 $GRAFT_REPO_ROOT/verkle-kzg_amd/tools/commit_ab.py 3 16:15 > $GRAFT_REPO_ROOT/$O/write.log 2>&1 || exit $?
