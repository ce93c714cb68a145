#!/bin/bash
# Build a libcvq.so variant with extra -D flags on the COMPACT translation units (CPU container).
# usage: tools/build_variant_compact.sh <name> <flags...>   -> build_variants/<name>/libcvq.so
# The other objects come from the package's build/ (brought up to date by make first, so a
# variant never links an object compiled from older headers).  With -DCVQ_DEV_CFG2 only
# cfg 2's slice (Student, MSM, nu = 6) holds kernels, and the build takes seconds.
set -e
name=$1; shift
cd "$(dirname "$0")/../copula-msm-and-copula-garch-var_amd"
flock /tmp/cvq_make.lock make -s build/cvq_plan.o build/cvq_forecast.o build/cvq_sorted.o
out=../build_variants/$name
mkdir -p $out
CXX="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
$CXX "$@" -c csrc/cvq_compact.hip -o $out/cvq_compact.o
objs=""; pids=""
for s in st_msm_8 st_msm_0 st_gar_8 st_gar_0 ga_msm ga_gar pl_msm pl_gar; do
  if [ "$s" = st_msm_8 ]; then
    $CXX "$@" -DCVQ_INST_$s -c csrc/cvq_compact_inst.hip -o $out/cvq_ci_$s.o -Rpass-analysis=kernel-resource-usage \
        2> $out/resource.txt &
    pids="$pids $!"
  else
    $CXX "$@" -DCVQ_INST_$s -c csrc/cvq_compact_inst.hip -o $out/cvq_ci_$s.o &
    pids="$pids $!"
  fi
  objs="$objs $out/cvq_ci_$s.o"
done
for p in $pids; do wait $p; done        # set -e: a failed slice stops the script
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libcvq.so build/cvq_plan.o build/cvq_forecast.o \
    $out/cvq_compact.o build/cvq_sorted.o build/cvq_si_*.o $objs
