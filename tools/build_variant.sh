#!/bin/bash
# Build a libkp variant with extra -D flags into tools/variants/<name>/libkp.so (KP_LIB selects it): both kernel
# translation units as the Makefile builds them (KP_TU 1 with the ILP scheduler, KP_TU 2 default), plus the flags.
# usage: build_variant.sh <name> [-DFLAG=1 ...]
set -e
name=$1; shift
cd "$(dirname "$0")/../karpenter-provider-aws_amd"
mkdir -p ../tools/variants/$name build
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -include ../tools/kp_diag.h -Wno-unused-function"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=max-ilp -DKP_TU=1 "$@" -c csrc/kp_kernels.hip -o build/kp_kernels_$name.o
/opt/rocm/bin/hipcc $F -DKP_TU=2 "$@" -c csrc/kp_kernels.hip -o build/kp_filter_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/variants/$name/libkp.so.tmp build/kp_kernels_$name.o build/kp_filter_$name.o build/kp_host.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && mv -f ../tools/variants/$name/libkp.so.tmp ../tools/variants/$name/libkp.so
