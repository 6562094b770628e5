#!/bin/bash
# SQ counters of the tick kernels on C4 and on C2 at 2^22 groups, the
# counter list, and C4 without isolation windows (timing reference)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3sq}
mkdir -p $OUT
P="timeout -s KILL 120 rocprofv3"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
C4="--workload C4 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline"
C24="--workload C2 --groups-per-gpu 4194304 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline"
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
$P --pmc $SQ -d $OUT/sq_c4 -o p --output-format csv -- python3 -u bench.py $C4 > $OUT/sq1.log 2>&1 \
&& $P --pmc $SQ -d $OUT/sq_c24 -o p --output-format csv -- python3 -u bench.py $C24 > $OUT/sq2.log 2>&1 \
&& timeout -k 10 300 python3 -u bench.py --workload C4 --isolate 0 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4_noiso.json 2> $OUT/noiso.err \
&& timeout -k 10 300 python3 -u bench.py --workload C2 --groups-per-gpu 4194304 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c2_4m.json 2> $OUT/c24.err
