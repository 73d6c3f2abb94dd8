# the N = 4 flow on one card (window split from 4 ranks, host-callback exchange): bench.py starts its ranks itself
set -eu
R=$(pwd)
O=$R/gpurun_out/r06_rehearse4; mkdir -p $O
timeout -k 10 1000 python -u bench.py --gpus 4 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline > $O/rehearse_4rank.json 2> $O/rehearse_4rank.err
echo rehearse-done; tail -2 $O/rehearse_4rank.err
