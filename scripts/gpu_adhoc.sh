set -eu
R=$(pwd)
O=$R/gpurun_out/r06_smalltags; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scheme.py tests/test_gpu_verkle.py tests/test_gpu_verkle32.py tests/test_gpu_multiproof_256.py -m gpu > $O/tests_default.txt 2>&1
echo tests-default; tail -1 $O/tests_default.txt
VKZG_SMALL_TAGS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scheme.py tests/test_gpu_verkle.py tests/test_gpu_verkle32.py tests/test_gpu_multiproof_256.py -m gpu > $O/tests_tags.txt 2>&1
echo tests-tags; tail -1 $O/tests_tags.txt
bash scripts/ab_probe.sh $O/ab_ipa VKZG_SMALL_TAGS "1 0" 3 120 python -u verkle-kzg_amd/tools/ipa_abi_probe.py
VKZG_AB_FB_C=16 bash scripts/ab_probe.sh $O/ab_verkle VKZG_SMALL_TAGS "1 0" 3 180 python -u verkle-kzg_amd/tools/verkle_ab.py 65536 8
