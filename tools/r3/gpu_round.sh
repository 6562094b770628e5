#!/bin/bash
# One GPU session: full suite + bench lines (gpu_full.sh), an interleaved C4
# A/B against ablib builds (LIBS), C4's list size sweep, timing-only list
# kernel diagnostics (RAFTSTEP_DIAG_LEAN in LDIAGS), and a kernel trace of C4.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=${OUTDIR:-r3round}
OUT=gpurun_out/$O
mkdir -p $OUT
OUTDIR=$O bash tools/r3/gpu_full.sh || exit 1
[ -n "$LIBS" ] && { OUTDIR=$O WL=C4 ROUNDS=${ROUNDS:-2} bash tools/r3/gpu_try.sh || exit 1; }
for i in $SWEEP; do
  timeout -k 10 300 python -u bench.py --workload C4 --isolate $i --steps 20 --warmup 5 --no-cpu-baseline \
    > $OUT/c4_iso$i.json 2> $OUT/c4_iso$i.err || exit 1
done
for v in $LDIAGS; do
  RAFTSTEP_DIAG_LEAN=$v timeout -k 10 300 python -u bench.py --workload C4 --steps 20 --warmup 5 --repeats 3 \
    --no-cpu-baseline > $OUT/c4_ldiag$v.json 2> $OUT/c4_ldiag$v.err
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c4 --output-format csv -- python3 -u bench.py \
  --workload C4 --steps 20 --warmup 5 --repeats 2 --no-cpu-baseline > $OUT/kt.log 2>&1 || exit 1
exit 0
