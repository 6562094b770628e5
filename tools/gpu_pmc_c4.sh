#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) over the C4 bench, to
# attribute per-launch HBM traffic of the fast and general kernels.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python3 -u bench.py --workload C4 --steps 24 --warmup 2 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_c4_fetch -o p --output-format csv -- $B > $OUT/pmc_c4_1.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_c4_write -o p --output-format csv -- $B > $OUT/pmc_c4_2.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T -d $OUT/pmc_c4_sq -o p --output-format csv -- $B > $OUT/pmc_c4_3.log 2>&1
