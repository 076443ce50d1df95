#!/bin/bash
# Diagnostic FT_FINE build of libkp (the fast-lane phase probes, finer ones included) into tools/fine/libkp.so (KP_LIB=... selects it).
set -e
cd "$(dirname "$0")/../karpenter-provider-aws_amd"
mkdir -p ../tools/fine build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -include ../tools/kp_diag.h -Wno-unused-function -mllvm -amdgpu-sched-strategy=max-ilp -DKP_TU=1 -DFT_FINE=1 -DFL_NOTIME=0 -c csrc/kp_kernels.hip -o build/kp_kernels_fine.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/fine/libkp.so.tmp build/kp_kernels_fine.o build/kp_filter.o build/kp_host.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && mv -f ../tools/fine/libkp.so.tmp ../tools/fine/libkp.so
