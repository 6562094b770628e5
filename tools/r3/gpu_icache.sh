#!/bin/bash
# Instruction-side counters of the C4 tick kernels: is the list kernel
# (8.9K instructions, one wave per SIMD) bound by instruction fetch?
# counters.txt lists what this rocprofv3 offers.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3ic}
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
C4="--workload C4 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline"
pass() {   # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 -u bench.py $C4 \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $OUT/progress.log
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
pass sq_inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_IFETCH SQ_WAIT_INST_LDS
pass sqc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES
pass sq_wait SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC
exit 0
