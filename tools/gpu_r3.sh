#!/bin/bash
# Round 3: new GPU tests first (-k filter via PYTEST_K), then optionally the
# whole GPU suite (FULL=1) and the bench lines at the driver's protocol
# (--steps 20 --warmup 5), each step under its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 600 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.log 2>&1 || exit 1
fi
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
&& timeout -k 10 300 python -u bench.py --workload C4 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err
