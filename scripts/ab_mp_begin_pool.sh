# A/B of the single multiproof's overlapped transcript filling (VKZG_MP_BEGIN_POOL 1 / 0), 3
# alternating rounds of the bench's multiproof line
set -o pipefail
O=${1:-gpurun_out/mp_begin_pool}
mkdir -p $O
for r in 1 2 3; do for v in 1 0; do
  timeout -k 10 200 env VKZG_MP_BEGIN_POOL=$v python -u bench.py --steps 3 --warmup 1 --log-n 16 --no-secondary --no-kzg --no-verkle --no-ipa --no-cpu-baseline --no-variable-base --no-check > $O/r${r}_pool$v.json 2>/dev/null || exit $?
done; done
