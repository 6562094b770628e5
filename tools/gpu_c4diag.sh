#!/bin/bash
# Parity suite, then C4 diagnostics: general-kernel worklist size per launch
# and fast-kernel lane classes with deferral reasons (both synchronising, so
# not timing runs), then plain C2 and C4 bench lines. The reason counters are
# compiled only into a diagnostics build: on the CPU side first run
#   touch raft-sample_amd/csrc/k_fast.hip && make -C raft-sample_amd/csrc DIAG=1
# (and rebuild without DIAG=1 afterwards); a product build prints zeros there.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& RAFTSTEP_DEBUG_WORK=1 timeout -k 10 200 python3 -u bench.py --workload C4 --steps 64 --warmup 16 --no-cpu-baseline > $OUT/c4_work.log 2>&1 \
&& RAFTSTEP_DEBUG_FAST=1 timeout -k 10 200 python3 -u bench.py --workload C4 --steps 64 --warmup 16 --no-cpu-baseline > $OUT/c4_fast.log 2>&1 \
&& timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/c2_bench.log 2>&1 \
&& timeout -k 10 200 python3 -u bench.py --workload C4 --steps 100 --warmup 16 --no-cpu-baseline > $OUT/c4_bench.log 2>&1
