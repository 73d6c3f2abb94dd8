#!/bin/bash
# round-3 probe batch 23: long fix-up chains split off (VKZG_FIXUP_LONG A/B), then the bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3z}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_comm.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py > $O/tests_full.txt 2>&1 || exit 1
P=verkle-kzg_amd/tools/msm_probe.py
for k in 1 2; do
for m in 0 1; do
VKZG_FIXUP_LONG=$m timeout -k 10 120 python -u $P bls12_381 20 > $O/radix_l${m}_$k.txt 2>&1 || exit 1
done
done
timeout -k 10 120 python -u verkle-kzg_amd/tools/adversarial_probe.py > $O/adversarial.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
