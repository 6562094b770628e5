#!/bin/bash
# GPU tests (TESTS), then an interleaved A/B of environment settings on one
# build: for each round, the default run and one per VARIANTS entry
# ("name:VAR=value,VAR2=value"), workload WL, driver protocol.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3envab}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || exit 1
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in cur $VARIANTS; do
    name=${v%%:*}; envs=""
    [ "$v" != "cur" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
    env $envs timeout -k 10 300 python -u bench.py --workload ${WL:-C4} --steps 20 --warmup 5 --no-cpu-baseline \
      > $OUT/bench_${WL:-C4}_${name}_$i.json 2> $OUT/bench_${WL:-C4}_${name}_$i.err || exit 1
  done
done
