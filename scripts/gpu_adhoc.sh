set -eu
R=$(pwd)
O=$R/gpurun_out/r06_mpomp; mkdir -p $O
timeout -k 10 300 python -u verkle-kzg_amd/tools/mp_phase_probe.py 16 12 > $O/default.txt 2>&1
OMP_WAIT_POLICY=PASSIVE timeout -k 10 300 python -u verkle-kzg_amd/tools/mp_phase_probe.py 16 12 > $O/omp_passive.txt 2>&1
timeout -k 10 300 python -u verkle-kzg_amd/tools/mp_phase_probe.py 16 12 > $O/default2.txt 2>&1
echo done
