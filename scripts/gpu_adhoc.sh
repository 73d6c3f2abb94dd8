set -eu
O=gpurun_out/r06_e; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_verkle32.py tests/test_gpu_verkle.py -k "verkle32 or update_equals" > $O/tests.txt 2>&1
echo tests-ok; tail -2 $O/tests.txt
timeout -k 10 300 python -u verkle-kzg_amd/tools/verkle_update_check.py 65536 5 91 0 > $O/update_check.txt 2>&1
echo check-ok; tail -5 $O/update_check.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-secondary --no-kzg --no-mp --no-ipa > $O/bench_verkle.json 2> $O/bench_verkle.err
echo bench-ok
timeout -k 10 300 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-kzg --no-mp --no-ipa --no-verkle > $O/rehearse_2rank.json 2> $O/rehearse_2rank.err
echo rehearse-ok
