#!/bin/bash
# Build a libcvq.so variant with extra -D flags on the COMPACT translation unit (CPU container).
# usage: tools/build_variant_compact.sh <name> <flags...>   -> build_variants/<name>/libcvq.so
# The other objects come from the package's build/ (brought up to date by make first, so a
# variant never links an object compiled from older headers).
set -e
name=$1; shift
cd "$(dirname "$0")/../copula-msm-and-copula-garch-var_amd"
flock /tmp/cvq_make.lock make -s build/cvq_plan.o build/cvq_forecast.o build/cvq_sorted.o
out=../build_variants/$name
mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function "$@" \
    -c csrc/cvq_compact.hip -o $out/cvq_compact.o -Rpass-analysis=kernel-resource-usage 2> $out/resource.txt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libcvq.so build/cvq_plan.o build/cvq_forecast.o \
    $out/cvq_compact.o build/cvq_sorted.o
