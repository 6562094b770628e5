#!/bin/bash
# Two-pass plan diagnostics on C4: lean-only floor (no isolation), single-pass
# A/B, and FETCH_SIZE / WRITE_SIZE passes over both kernels of the two-pass tick.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2tp}
mkdir -p $OUT
B="python3 -u bench.py"
C4="--workload C4 --steps 24 --warmup 4 --repeats 1 --no-cpu-baseline"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step noiso && timeout -k 10 200 $B --workload C4 --isolate 0 --steps 64 --warmup 16 --repeats 3 --no-cpu-baseline > $OUT/c4_noiso.log 2>&1 \
&& step single && RAFTSTEP_TWO_PASS=0 timeout -k 10 200 $B --workload C4 --steps 64 --warmup 16 --repeats 3 --no-cpu-baseline > $OUT/c4_single.log 2>&1 \
&& step fetch && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_c4_fetch -o p --output-format csv -- python3 -u bench.py $C4 > $OUT/pmc1.log 2>&1 \
&& step write && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_c4_write -o p --output-format csv -- python3 -u bench.py $C4 > $OUT/pmc2.log 2>&1 \
&& step fetch1 && RAFTSTEP_TWO_PASS=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_c4s_fetch -o p --output-format csv -- python3 -u bench.py $C4 > $OUT/pmc3.log 2>&1 \
&& step write1 && RAFTSTEP_TWO_PASS=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_c4s_write -o p --output-format csv -- python3 -u bench.py $C4 > $OUT/pmc4.log 2>&1 \
&& step done
