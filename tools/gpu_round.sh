#!/bin/bash
# One GPU session: parity tests, benches, kernel-trace profile. Each GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-200}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& timeout -k 10 240 python -u bench.py --steps $STEPS --warmup 20 > $OUT/bench.log 2>&1 \
&& timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --groups-per-gpu 4194304 --no-cpu-baseline > $OUT/bench_4m.log 2>&1 \
&& timeout -k 10 240 python -u bench.py --workload C5 --steps 30 --warmup 3 > $OUT/bench_c5.log 2>&1 \
&& timeout -k 10 180 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o run --output-format csv -- python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1
