# round-end rehearsal, part 2 of 2 (scripts/round_final.sh's second half): the bench line with the
# installed counters, the self-launched two-rank flow on one card, the one-card split probe
set -eu
R=$(pwd)
O=$R/gpurun_out/r06_final4; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
echo bench-done; tail -3 $O/bench.err
timeout -k 10 600 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline > $O/rehearse_2rank.json 2> $O/rehearse_2rank.err
echo rehearse-done
timeout -k 10 300 python -u verkle-kzg_amd/tools/split_probe.py 1,2,8 > $O/split_probe.txt 2>&1
echo split-done
