#!/bin/bash
# Interleaved A/B of the round-2 build (ablib/r2tree: its bench.py, Python
# binding and library, built from ff5c4c4) against this tree, on WORKLOADS.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${OUTDIR:-r4r2}
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for w in ${WORKLOADS:-C4R C4}; do
    echo "== $(date +%T) round $r $w r2" >> "$OUT/progress.log"
    (cd ablib/r2tree && timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline) \
      > "$OUT/r2_${w}_$r.json" 2> "$OUT/r2_${w}_$r.err" || exit 1
    echo "== $(date +%T) round $r $w cur" >> "$OUT/progress.log"
    timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-fused --extra none \
      > "$OUT/cur_${w}_$r.json" 2> "$OUT/cur_${w}_$r.err" || exit 1
  done
done
echo "== $(date +%T) done" >> "$OUT/progress.log"
