#!/bin/bash
# Build a libcvq.so variant with extra -D flags on the forecast translation unit (CPU container).
# usage: tools/build_variant_forecast.sh <name> <flags...>   -> build_variants/<name>/libcvq.so
set -e
name=$1; shift
cd "$(dirname "$0")/../copula-msm-and-copula-garch-var_amd"
flock /tmp/cvq_make.lock make -s
out=../build_variants/$name
mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function "$@" \
    -c csrc/cvq_forecast.hip -o $out/cvq_forecast.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libcvq.so build/cvq_plan.o $out/cvq_forecast.o \
    build/cvq_compact.o build/cvq_sorted.o build/cvq_ci_*.o build/cvq_si_*.o
