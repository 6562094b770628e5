#!/bin/bash
# timing-only A/B of the lean kernel's write-pattern diagnostics on C4
# (RAFTSTEP_DIAG_LEAN: 4 = no holes, 8 = no stale-column writes); the
# diagnosed runs' results are wrong by design (their stats check may fail)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUTDIR:-r3ab}
mkdir -p $OUT
for dl in ${DIAGS:-0 4 8 12 0}; do
  RAFTSTEP_DIAG_LEAN=$dl timeout -k 10 300 python -u bench.py --workload ${WL:-C4} --steps 20 --warmup 5 --no-cpu-baseline \
    > $OUT/bench_diag$dl.json 2> $OUT/bench_diag$dl.err || true
done
