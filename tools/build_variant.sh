#!/bin/bash
# build an ablation/tuning variant of libqe: tools/build_variant.sh NAME "-DFLAG=V ..."
set -e
cd "$(dirname "$0")/../query-compiler-executor_amd"
# objects in build/diag (gpurun-ignored); the library in build/var, which gpurun ships -- delete it
# after its A/B (every call pushes it)
out=build/diag/$1; rm -rf $out; mkdir -p $out build/var
pids=()
for f in csrc/*.hip; do /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I../include -munsafe-fp-atomics $2 -c $f -o $out/$(basename $f .hip).o & pids+=($!); done
for p in "${pids[@]}"; do wait $p; done   # any failed compile fails the script
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o build/var/libqe_$1.so $out/*.o build/qe_exec.o build/qe_query.o build/qe_plan.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built build/var/libqe_$1.so
