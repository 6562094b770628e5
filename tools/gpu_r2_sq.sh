#!/bin/bash
# One SQ counter pass over a short C4 run (wave cycles busy / waiting,
# instruction mix per kernel); WL / ARGS select another workload.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2sq}
mkdir -p $OUT
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
timeout -s KILL 120 rocprofv3 --pmc $SQ -T -d $OUT/sq -o p --output-format csv -- python3 -u bench.py --workload ${WL:-C4} --steps 24 --warmup 4 --repeats 1 --no-cpu-baseline > $OUT/sq.log 2>&1
