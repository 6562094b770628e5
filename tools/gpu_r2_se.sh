#!/bin/bash
# C4 vs the general kernel's cadence (RAFTSTEP_SLOW_EVERY), interleaved,
# plus the worklist per launch at cadence 1 and a kernel trace at 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2se}
mkdir -p $OUT
B="python3 -u bench.py --no-cpu-baseline --workload C4 --steps 64 --warmup 200 --repeats 3"
for se in 8 1 2 4 16 8 1; do
  echo "== $(date +%T) se $se" >> $OUT/progress.log
  RAFTSTEP_SLOW_EVERY=$se timeout -k 10 200 $B >> $OUT/c4_se$se.log 2>&1 || exit 1
done
RAFTSTEP_SLOW_EVERY=1 RAFTSTEP_DEBUG_WORK=1 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --workload C4 --steps 16 --warmup 200 --repeats 1 > $OUT/c4_se1_work.log 2>&1 \
&& RAFTSTEP_SLOW_EVERY=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_se1 -o run --output-format csv -- python3 -u bench.py --workload C4 --steps 32 --warmup 200 --repeats 1 --no-cpu-baseline > $OUT/prof_se1.log 2>&1
