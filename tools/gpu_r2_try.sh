#!/bin/bash
# Iteration loop: the RAFT / audit / KAT GPU tests first (PYTEST_K selects),
# then C4 bench lines and the deferral reasons (diaglib/).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2try}
mkdir -p $OUT
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step tests && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.log 2>&1 \
&& step c4 && timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --workload C4 --steps 64 --warmup 200 --repeats 3 > $OUT/c4.log 2>&1 \
&& step c4r && timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --workload C4R --steps 64 --warmup 200 --repeats 3 > $OUT/c4r.log 2>&1 \
&& step reasons && RAFTSTEP_LIB=diaglib/libraftstep_diag.so RAFTSTEP_DEBUG_FAST=1 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --workload C4 --steps 32 --warmup 200 --repeats 1 > $OUT/c4_reasons.log 2>&1 \
&& { [ -z "$SQ" ] || { step sq && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR -T -d $OUT/sq_c4 -o p --output-format csv -- python3 -u bench.py --workload C4 --steps 24 --warmup 200 --repeats 1 --no-cpu-baseline > $OUT/sq.log 2>&1; }; } \
&& step done
