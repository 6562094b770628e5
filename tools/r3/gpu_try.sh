#!/bin/bash
# A change on the GPU: GPU tests (TESTS, optional PYTEST_K filter), then an
# interleaved A/B of the in-tree build against ablib/libraftstep_<v>.so for
# each v in LIBS on workload WL (default C4), ROUNDS rounds, driver protocol.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3try}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.log 2>&1 || exit 1
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in cur ${LIBS:-prev}; do
    if [ $v = cur ]; then unset RAFTSTEP_LIB; else export RAFTSTEP_LIB=$PWD/ablib/libraftstep_$v.so; fi
    for wl in ${WL:-C4}; do   # a workload name, or name:groups
      G=""; [ "${wl#*:}" != "$wl" ] && G="--groups-per-gpu ${wl#*:}"
      timeout -k 10 300 python -u bench.py --workload ${wl%%:*} $G --steps 20 --warmup 5 --no-cpu-baseline \
        > $OUT/bench_${wl/:/_}_${v}_$i.json 2> $OUT/bench_${wl/:/_}_${v}_$i.err || exit 1
    done
  done
done
# timing-only lean-kernel diagnostics (RAFTSTEP_DIAG_LEAN values in DIAGS) on C2 at 2^22 groups and on C4
for v in $DIAGS; do
  RAFTSTEP_DIAG_LEAN=$v timeout -k 10 300 python -u bench.py --workload C2 --groups-per-gpu 4194304 --steps 20 --warmup 5 \
    --repeats 3 --no-cpu-baseline > $OUT/c2_4m_diag$v.json 2> $OUT/c2_4m_diag$v.err
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  RAFTSTEP_DIAG_LEAN=$v timeout -k 10 300 python -u bench.py --workload C4 --steps 20 --warmup 5 \
    --repeats 3 --no-cpu-baseline > $OUT/c4_diag$v.json 2> $OUT/c4_diag$v.err
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
