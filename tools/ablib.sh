#!/bin/bash
# Builds an A/B variant of libraftstep.so with extra compile-time flags into
# ablib/<name>/ (bench.py / tests pick it with RAFTSTEP_LIB=ablib/<name>/libraftstep.so).
#   tools/ablib.sh la32 -DRAFTSTEP_LIST_LANES=32
# ablib/ is in .gpurunignore (it never travels with the snapshot): build the
# variants ON the GPU box, inside the gpurun command (tools/gpu_ab.sh does).
set -e
name=$1; shift
cd "$(dirname "$0")/../raft-sample_amd/csrc"
out=../../ablib/$name
mkdir -p "$out"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
pids=()
for f in k_fast k_ref k_raft k_init; do /opt/rocm/bin/hipcc $F -c $f.hip -o "$out/$f.o" & pids+=($!); done
/opt/rocm/bin/hipcc $F -c engine.cpp -o "$out/engine.o" & pids+=($!)
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out/libraftstep.so" "$out"/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f "$out"/*.o
echo "built $out/libraftstep.so ($*)"
