#!/bin/bash
# Build an A/B variant of libmipipe.so from a modified copy of csrc/ (CPU side, before a GPU call).
# usage: build_variant.sh <variant-csrc-dir> <out-name.so>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; OUT=$R/distributed-llm-pipeline_amd/lib/$2
B=$(mktemp -d); trap 'rm -rf $B' EXIT
FL="-std=c++17 -O3 -fPIC -I/opt/rocm/include -I$SRC/runtime --offload-arch=gfx950"
pids=()
for f in $SRC/kernels/*.hip; do /opt/rocm/bin/hipcc $FL -munsafe-fp-atomics -c $f -o $B/k_$(basename $f .hip).o & pids+=($!); done
for f in $SRC/runtime/*.cpp; do /opt/rocm/bin/hipcc $FL -D__HIP_PLATFORM_AMD__ -c $f -o $B/r_$(basename $f .cpp).o & pids+=($!); done
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT $B/*.o -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
echo "built $OUT"
