#!/bin/bash
# Stall attribution of the C4 general kernel: instruction-cache and wait counters.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python3 -u bench.py --workload C4 --steps 24 --warmup 2 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY -T -d $OUT/pmc_c4_stall -o p --output-format csv -- $B > $OUT/pmc_c4_4.log 2>&1
