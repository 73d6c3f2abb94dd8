# a second bench line on the round's final library (box-to-box spread; bench.py as the driver runs it)
set -eu
R=$(pwd)
O=$R/gpurun_out/r06_final8b; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
echo bench-done; tail -2 $O/bench.err
