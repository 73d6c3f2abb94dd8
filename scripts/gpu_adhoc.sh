set -eu
R=$(pwd)
O=$R/gpurun_out/r06_xinline; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scheme.py tests/test_gpu_multiproof_256.py tests/test_gpu_fullsize.py -m gpu > $O/tests.txt 2>&1
echo tests; tail -1 $O/tests.txt
bash scripts/ab_probe.sh $O/ab VKZG_IPA_X_INLINE "1 0" 3 120 python -u verkle-kzg_amd/tools/ipa_abi_probe.py
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
VKZG_IPA_X_INLINE=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o run -- python3 -u $R/verkle-kzg_amd/tools/ipa_abi_probe.py > $O/trace_run_$v.txt 2>&1
done
echo done
