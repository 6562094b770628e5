#!/bin/bash
# Where C4's tick goes under the two-pass plan: lane classes
# (RAFTSTEP_DEBUG_FAST), C4 without isolation, the C2 shape at C4's size
# (4M x R=7, K=128: the lean kernel's floor), and rocprofv3 kernel-trace
# summaries of C4 and C2. Each GPU step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2look}
mkdir -p $OUT
B="python3 -u bench.py --no-cpu-baseline"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step diag && RAFTSTEP_DEBUG_FAST=1 timeout -k 10 200 $B --workload C4 --steps 32 --warmup 16 --repeats 1 > $OUT/c4_diag.log 2>&1 \
&& step noiso && timeout -k 10 200 $B --workload C4 --isolate 0 --steps 64 --warmup 16 --repeats 3 > $OUT/c4_noiso.log 2>&1 \
&& step c2r7 && timeout -k 10 200 $B --groups-per-gpu 4194304 --replicas 7 --ring-depth 128 --steps 64 --repeats 3 > $OUT/c2_4m_r7_k128.log 2>&1 \
&& step prof_c4 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c4 -o run --output-format csv -- python3 -u bench.py --workload C4 --steps 64 --warmup 16 --repeats 1 --no-cpu-baseline > $OUT/prof_c4.log 2>&1 \
&& step prof_c2 && timeout -k 10 180 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c2 -o run --output-format csv -- python3 -u bench.py --steps 200 --warmup 20 --repeats 1 --no-cpu-baseline > $OUT/prof_c2.log 2>&1 \
&& step done
