#!/bin/bash
# round 5 step R: host EC / field operation timings on the GPU box's CPU, plain vs -mbmi2 -madx
set -u
O=gpurun_out/r05_r
mkdir -p $O
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -x hip --offload-arch=gfx950"
$H verkle-kzg_amd/tools/hostops.cpp -o /tmp/ho_a && $H -Xarch_host -mbmi2 -Xarch_host -madx verkle-kzg_amd/tools/hostops.cpp -o /tmp/ho_b || exit 1
for k in 1 2; do echo "plain:" >> $O/hostops.txt; /tmp/ho_a >> $O/hostops.txt; echo "bmi2+adx:" >> $O/hostops.txt; /tmp/ho_b >> $O/hostops.txt; done
cat $O/hostops.txt
