#!/bin/bash
# round-3 probe batch 22: tests + headline after the one-round rule of the marginal bit stage;
# instruction-fetch / wait counters of the tail kernels (are they code-fetch bound?)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3z}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_comm.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py > $O/tests_full.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
timeout -k 10 120 python -u $P bls12_381 20 > $O/radix.txt 2>&1 || exit 1
VKZG_MSM_SHARED=0 timeout -k 10 120 python -u $P bls12_381 20 > $O/vb.txt 2>&1 || exit 1
timeout -k 10 120 python -u $P bn254 20 > $O/bn254.txt 2>&1 || exit 1
timeout -k 10 200 python -u verkle-kzg_amd/tools/scale_probe.py > $O/scale.txt 2>&1 || exit 1
Q=verkle-kzg_amd/tools/msm_once.py
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_INSTS_VALU -d $O/pmc1 -o pmc1 --output-format csv -- python3 $Q bls12_381 20 3 > $O/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES -d $O/pmc2 -o pmc2 --output-format csv -- python3 $Q bls12_381 20 3 > $O/pmc2.log 2>&1 || exit 1
