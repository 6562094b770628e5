#!/bin/bash
# PMC passes (one counter group per run, per MI355X_MICROARCH.md) + A/B.
# Each step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 python3 -u tools/ab.py --ticks 100 --rounds 5 base: wt:RAFTSTEP_WRITE_THROUGH=1 se32:RAFTSTEP_SLOW_EVERY=32 > $OUT/ab.log 2>&1 \
&& timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_calib_fetch -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc1.log 2>&1 \
&& timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_calib_write -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc2.log 2>&1 \
&& timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_fetch -o p --output-format csv -- $B > $OUT/pmc3.log 2>&1 \
&& timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_write -o p --output-format csv -- $B > $OUT/pmc4.log 2>&1 \
&& timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -T -d $OUT/pmc_sq -o p --output-format csv -- $B > $OUT/pmc5.log 2>&1
