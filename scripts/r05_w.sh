#!/bin/bash
# round 5 step W: window bits of the lazily built fixed-base tables (the IPA CRS, multiproof D / E):
# VKZG_FB_C_DEFAULT 8 / 12 / 16 -- IPA prove / verify and the multiproof finish
set -u
O=gpurun_out/r05_w
mkdir -p $O
export TMPDIR=/tmp
bash scripts/ab_probe.sh $O VKZG_FB_C_DEFAULT "8 12 16" 2 200 python -u verkle-kzg_amd/tools/ipa_probe.py || exit $?
bash scripts/ab_probe.sh $O/mp VKZG_FB_C_DEFAULT "8 12 16" 2 200 python -u verkle-kzg_amd/tools/mp_probe.py 16 || exit $?
for f in $O/VKZG_FB_C_DEFAULT_*; do echo "$f: $(grep -E '^(prove|verify)' $f | tr '\n' ' ')"; done
for f in $O/mp/VKZG_FB_C_DEFAULT_*; do echo "$f: $(grep -E 'finish' $f | tail -2 | tr '\n' ' ')"; done
