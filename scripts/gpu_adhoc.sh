set -eu
R=$(pwd)
O=$R/gpurun_out/r06_final2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo tests-done; tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo smoke-done
bash $R/scripts/bench_profile.sh r06_final2
mkdir -p $O/profiles_r06 && cp $R/gpurun_out/prof_r06_final2/summary.json $O/profiles_r06/pmc_summary.json
echo profile-done
