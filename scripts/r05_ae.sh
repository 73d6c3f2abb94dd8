#!/bin/bash
# round 5 step AE: the Python mirror's proof marshalling (one buffer per proof, bulk integer
# conversion): scheme / multiproof / verkle / group / comm / threads GPU tests, then ipa_abi_probe.py
set -u
O=gpurun_out/r05_ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scheme.py tests/test_gpu_multiproof_256.py tests/test_gpu_verkle.py tests/test_gpu_group.py tests/test_gpu_comm.py tests/test_gpu_threads.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_abi_probe.py >> $O/probe.txt 2>&1 || exit $?; done
cat $O/probe.txt
