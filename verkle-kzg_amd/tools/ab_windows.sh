# same-box A/B: shared-window copies in radix-29 limbs (default) vs packed-29 (VKZG_WIN_PACKED=1)
set -e
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 3 --no-secondary --no-kzg --no-mp --no-verkle --no-ipa --no-cpu-baseline --no-variable-base"
for i in 1 2; do
timeout -k 10 120 $B > gpurun_out/ab_limbs_$i.json 2>/dev/null
VKZG_WIN_PACKED=1 timeout -k 10 120 $B > gpurun_out/ab_packed_$i.json 2>/dev/null
done
timeout -k 10 150 python verkle-kzg_amd/tools/commit_breakdown.py 16 > gpurun_out/commit_bd4.log 2>&1
