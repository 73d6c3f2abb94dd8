# round 5 step K: the bench's verkle call sequence, every update timed (with / without the timing tree)
set -u
O=gpurun_out/r05_k2
mkdir -p $O
for k in 1 0 1; do
  timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_bench_seq.py $k 6 >> $O/seq.txt 2>&1 || exit $?
done
VKZG_VERBOSE=1 timeout -k 10 200 python -u verkle-kzg_amd/tools/verkle_bench_seq.py 1 6 > $O/seq_laps.txt 2>&1 || exit $?
