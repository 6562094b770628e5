#!/bin/bash
# build ablib/libraftstep_head.so from HEAD's k_fast.hip (other objects as in tree) for an A/B
set -e
cd "$(dirname "$0")/../../raft-sample_amd/csrc"
git show HEAD:raft-sample_amd/csrc/k_fast.hip > /tmp/k_fast_head.hip
cp /tmp/k_fast_head.hip /tmp/kfh_dir_k_fast.hip
mkdir -p /tmp/kfh && cp *.hpp *.h *.inc /tmp/kfh/ && cp /tmp/k_fast_head.hip /tmp/kfh/k_fast.hip
mkdir -p /tmp/include && cp ../../include/raftstep.h /tmp/include/
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -c /tmp/kfh/k_fast.hip -o /tmp/k_fast_head.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../ablib/libraftstep_head.so /tmp/k_fast_head.o ../lib/k_ref.o ../lib/k_raft.o ../lib/k_init.o ../lib/engine.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
