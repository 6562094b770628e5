#!/bin/bash
# GPU tests (TESTS) then an interleaved A/B of the fused steady ticks
# (default RAFTSTEP_FUSE=4 vs 1) on C2, C2 at 2^22 and C3.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3fuse}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || exit 1
fi
for i in 1 2; do
  for f in 4 1; do
    RAFTSTEP_FUSE=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_f${f}_$i.json 2> $OUT/c2_f${f}_$i.err || exit 1
    RAFTSTEP_FUSE=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --groups-per-gpu 4194304 --no-cpu-baseline > $OUT/c2_4m_f${f}_$i.json 2> $OUT/c2_4m_f${f}_$i.err || exit 1
    RAFTSTEP_FUSE=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload C3 --no-cpu-baseline > $OUT/c3_f${f}_$i.json 2> $OUT/c3_f${f}_$i.err || exit 1
  done
done
