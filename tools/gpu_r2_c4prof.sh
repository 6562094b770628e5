#!/bin/bash
# C4 diagnostics: fast-kernel lane classes (RAFTSTEP_DEBUG_FAST), the same
# shape without isolation (the steady floor), and one SQ counter pass on
# C4 and on C2 (wave cycles: busy / waiting / issuing, instruction mix).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2c4p}
mkdir -p $OUT
B="python3 -u bench.py"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step diag && RAFTSTEP_DEBUG_FAST=1 timeout -k 10 200 $B --workload C4 --steps 32 --warmup 16 --repeats 1 --no-cpu-baseline > $OUT/c4_diag.log 2>&1 \
&& step noiso && timeout -k 10 200 $B --workload C4 --isolate 0 --steps 64 --warmup 16 --repeats 3 --no-cpu-baseline > $OUT/c4_noiso.log 2>&1 \
&& step c4 && timeout -k 10 200 $B --workload C4 --steps 64 --warmup 16 --repeats 3 --no-cpu-baseline > $OUT/c4.log 2>&1 \
&& step sq_c4 && timeout -s KILL 120 rocprofv3 --pmc $SQ -T -d $OUT/sq_c4 -o p --output-format csv -- python3 -u bench.py --workload C4 --steps 24 --warmup 4 --repeats 1 --no-cpu-baseline > $OUT/sq_c4.log 2>&1 \
&& step sq_c2 && timeout -s KILL 120 rocprofv3 --pmc $SQ -T -d $OUT/sq_c2 -o p --output-format csv -- python3 -u bench.py --steps 24 --warmup 4 --repeats 1 --no-cpu-baseline > $OUT/sq_c2.log 2>&1 \
&& step done
