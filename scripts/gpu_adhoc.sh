# second full parity run on the final library (another box)
set -eu
R=$(pwd)
O=$R/gpurun_out/r06_tests2; mkdir -p $O
sha256sum verkle-kzg_amd/lib/libvkzg.so > $O/lib_sha.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo tests-done; tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo smoke-done
