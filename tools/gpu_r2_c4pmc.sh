#!/bin/bash
# C4 under the two-pass plan: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate
# passes) and SQ wave-cycle counters of the lean and list kernels, with and
# without isolation; the pmc_calib passes for the FETCH/WRITE corrections.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2c4pmc}
mkdir -p $OUT
P="timeout -s KILL 120 rocprofv3"
C4A="--workload C4 --steps 24 --warmup 4 --repeats 1 --no-cpu-baseline"
C4N="--workload C4 --isolate 0 --steps 24 --warmup 4 --repeats 1 --no-cpu-baseline"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step calib && $P --pmc FETCH_SIZE -T -d $OUT/pmc_calib_fetch -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc1.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_calib_write -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc2.log 2>&1 \
&& step c4 && $P --pmc FETCH_SIZE -T -d $OUT/pmc_c4_fetch -o p --output-format csv -- python3 -u bench.py $C4A > $OUT/pmc3.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c4_write -o p --output-format csv -- python3 -u bench.py $C4A > $OUT/pmc4.log 2>&1 \
&& step c4n && $P --pmc FETCH_SIZE -T -d $OUT/pmc_c4n_fetch -o p --output-format csv -- python3 -u bench.py $C4N > $OUT/pmc5.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c4n_write -o p --output-format csv -- python3 -u bench.py $C4N > $OUT/pmc6.log 2>&1 \
&& step sq && $P --pmc $SQ -T -d $OUT/sq_c4 -o p --output-format csv -- python3 -u bench.py $C4A > $OUT/sq1.log 2>&1 \
&& $P --pmc $SQ -T -d $OUT/sq_c4n -o p --output-format csv -- python3 -u bench.py $C4N > $OUT/sq2.log 2>&1 \
&& step done
