#!/bin/bash
# C4 diagnostics in one call: per-tick lane classes of the timed region, then
# timing-only lean-kernel A/Bs (RAFTSTEP_DIAG_LEAN: 4 = no holes in the ring
# rows, 8 = no stale-column writes; results are wrong there, so a failed stats
# check, exit 1, is expected), and C4's shape without isolation (steady state).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3look}
mkdir -p $OUT
timeout -k 10 300 python -u tools/r3/class_probe.py C4 > $OUT/classes.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --workload C4 --steps 20 --warmup 5 --repeats 3"
for v in 0 4 8 12; do
  RAFTSTEP_DIAG_LEAN=$v timeout -k 10 300 $B > $OUT/c4_diag$v.json 2> $OUT/c4_diag$v.err
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "diag $v rc=$rc" >> $OUT/progress.log; exit $rc; fi
done
timeout -k 10 300 $B --isolate 0 > $OUT/c4_noiso.json 2> $OUT/c4_noiso.err || exit 1
# kernel trace of the C4 bench, then SQ counters of C4 and of C2 at 2^22 groups (one pass each)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c4 --output-format csv -- python3 -u bench.py --workload C4 --steps 20 --warmup 5 --repeats 2 --no-cpu-baseline > $OUT/kt.log 2>&1 || exit 1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR"
timeout -s KILL 120 rocprofv3 --pmc $SQ -d $OUT/sq_c4 -o p --output-format csv -- python3 -u bench.py --workload C4 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline > $OUT/sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $SQ -d $OUT/sq_c24 -o p --output-format csv -- python3 -u bench.py --workload C2 --groups-per-gpu 4194304 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline > $OUT/sq2.log 2>&1 || exit 1
