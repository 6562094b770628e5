#!/bin/bash
# rocprofv3 kernel-trace summary of one bench workload (WL), into OUT/prof
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2pf}
mkdir -p $OUT
WL=${WL:---workload C4 --steps 64 --warmup 16}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o run --output-format csv -- python3 -u bench.py $WL --repeats 1 --no-cpu-baseline > $OUT/prof.log 2>&1
