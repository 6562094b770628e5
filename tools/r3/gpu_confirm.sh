#!/bin/bash
# Confirmation of the committed defaults: the whole GPU suite, the driver's
# bench command, the other steady lines, C4, and a kernel trace of the C2 bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3conf}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
&& timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --groups-per-gpu 4194304 --no-cpu-baseline > $OUT/bench_c2_4m.json 2> $OUT/bench_c2_4m.err \
&& timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload C3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err \
&& timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload C4 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err \
&& timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --repeats 2 --no-cpu-baseline > $OUT/prof_c2.log 2>&1
