#!/bin/bash
# Build a libkp variant with extra -D flags into tools/variants/<name>/libkp.so (KP_LIB selects it).
# usage: build_variant.sh <name> [-DFLAG=1 ...]
set -e
name=$1; shift
cd "$(dirname "$0")/../karpenter-provider-aws_amd"
mkdir -p ../tools/variants/$name build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -Wno-unused-function "$@" -c csrc/kp_kernels.hip -o build/kp_kernels_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/variants/$name/libkp.so.tmp build/kp_kernels_$name.o build/kp_host.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && mv -f ../tools/variants/$name/libkp.so.tmp ../tools/variants/$name/libkp.so
