#!/bin/bash
# round-3 probe batch 18: staged coarse scatter for every digit source (variable-base, slices)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3y}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_comm.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py > $O/tests_full.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
for i in 1 2; do
VKZG_MSM_SHARED=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/vb_st$i.txt 2>&1 || exit 1
VKZG_MSM_SHARED=0 VKZG_SORT_CSTAGE=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/vb_direct$i.txt 2>&1 || exit 1
done
timeout -k 10 120 python -u $P bn254 20 > $O/bn254_st.txt 2>&1 || exit 1
VKZG_SORT_CSTAGE=0 timeout -k 10 120 python -u $P bn254 20 > $O/bn254_direct.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace8 -o run --output-format csv -- python3 $R/verkle-kzg_amd/tools/slice_trace.py > $O/trace8.txt 2>&1 || exit 1
