#!/bin/bash
# Timing-only A/B of C4's lean kernel: as built, drifted lanes skipping their
# ring writes (RAFTSTEP_DIAG_LEAN=1), drifted lanes writing the common row (=2).
# The diagnostic runs produce wrong rings, so a failed stats check (exit 1)
# is expected there; anything else stops the script.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2drift}
mkdir -p $OUT
B="python3 -u bench.py --no-cpu-baseline --workload C4 --steps 64 --warmup 200 --repeats 3"
for v in 0 1 2 0; do
  echo "== $(date +%T) diag $v" >> $OUT/progress.log
  RAFTSTEP_DIAG_LEAN=$v timeout -k 10 200 $B >> $OUT/c4_diag$v.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "rc=$rc" >> $OUT/progress.log; exit $rc; fi
done
