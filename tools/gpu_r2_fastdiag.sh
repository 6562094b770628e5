#!/bin/bash
# Round 2: what sets C4's steady-state kernel time — ring size (TLB reach),
# R=7, RAFT + isolation — against steady C2-shaped runs at the same scale.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r2fd
mkdir -p $OUT
B="timeout -k 10 300 python3 -u bench.py --steps 48 --warmup 16 --repeats 3 --no-cpu-baseline"
true \
\
&& $B --groups-per-gpu 4194304 --replicas 7 --ring-depth 128 > $OUT/c2_4m_r7_k128.log 2>&1 \
&& $B --groups-per-gpu 4194304 --replicas 7 --ring-depth 32 > $OUT/c2_4m_r7_k32.log 2>&1 \
&& $B --groups-per-gpu 4194304 > $OUT/c2_4m_r5_k32.log 2>&1
