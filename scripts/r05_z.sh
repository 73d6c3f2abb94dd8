#!/bin/bash
# round 5 step Z: host phases of the IPA prover on the final library (VKZG_HOST_TIMING=1)
set -u
O=gpurun_out/r05_z
mkdir -p $O
export TMPDIR=/tmp
VKZG_HOST_TIMING=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/ipa_probe.py > $O/ipa_host_timing.txt 2>&1 || exit $?
grep -E "ipa_prove\]" $O/ipa_host_timing.txt | tail -3
grep -E "fb_small" $O/ipa_host_timing.txt | tail -10
