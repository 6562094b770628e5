#!/bin/bash
# The whole GPU suite, then the fused-tick depth on C2 and C2 at 2^22 (RAFTSTEP_FUSE 4 / 8 / 16, interleaved).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3fs}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2; do
  for f in 4 8 16; do
    RAFTSTEP_FUSE=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_f${f}_$i.json 2> $OUT/c2_f${f}_$i.err || exit 1
    RAFTSTEP_FUSE=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --groups-per-gpu 4194304 --no-cpu-baseline > $OUT/c2_4m_f${f}_$i.json 2> $OUT/c2_4m_f${f}_$i.err || exit 1
  done
done
