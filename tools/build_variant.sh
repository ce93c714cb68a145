#!/bin/bash
# Build a libcvq.so variant with extra -D flags on the SORTED translation units (CPU container).
# usage: tools/build_variant.sh <name> <flags...>   -> build_variants/<name>/libcvq.so
set -e
name=$1; shift
cd "$(dirname "$0")/../copula-msm-and-copula-garch-var_amd"
flock /tmp/cvq_make.lock make -s   # every base object up to date
out=../build_variants/$name
mkdir -p $out
CXX="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
$CXX "$@" -c csrc/cvq_sorted.hip -o $out/cvq_sorted.o &
for w in 384 512 1024; do
  $CXX "$@" -DCVQ_SORT_SLICE_$w -c csrc/cvq_sorted_inst.hip -o $out/cvq_si_$w.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libcvq.so build/cvq_plan.o build/cvq_forecast.o \
    build/cvq_compact.o build/cvq_ci_*.o $out/cvq_sorted.o $out/cvq_si_384.o $out/cvq_si_512.o $out/cvq_si_1024.o
