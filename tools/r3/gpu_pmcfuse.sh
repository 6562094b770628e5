#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (calibrated by tools/pmc_calib) of the fused
# steady lines at the default depth (16 ticks per launch): C2, C2 at 2^22, C3,
# with their bench lines (driver protocol) and a kernel trace of C2. Then
#   python tools/r3/summarize_evidence.py gpurun_out/r3pmcf pmc_fuse16 <commit>
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3pmcf}
mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 5"
P="timeout -s KILL 120 rocprofv3"
Q="--steps 20 --warmup 5 --repeats 1 --no-cpu-baseline"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step c2 && timeout -k 10 300 $B > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
&& step c2_4m && timeout -k 10 300 $B --groups-per-gpu 4194304 --no-cpu-baseline > $OUT/bench_c2_4m.json 2> $OUT/bench_c2_4m.err \
&& step c3 && timeout -k 10 300 $B --workload C3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err \
&& step prof_c2 && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 -u bench.py $Q > $OUT/prof_c2.log 2>&1 \
&& step pmc && $P --pmc FETCH_SIZE -d $OUT/pmc_calib_fetch -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc1.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_calib_write -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc2.log 2>&1 \
&& $P --pmc FETCH_SIZE -d $OUT/pmc_c2_fetch -o p --output-format csv -- python3 -u bench.py $Q > $OUT/pmc3.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_c2_write -o p --output-format csv -- python3 -u bench.py $Q > $OUT/pmc4.log 2>&1 \
&& $P --pmc FETCH_SIZE -d $OUT/pmc_c2_4m_fetch -o p --output-format csv -- python3 -u bench.py --groups-per-gpu 4194304 $Q > $OUT/pmc5.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_c2_4m_write -o p --output-format csv -- python3 -u bench.py --groups-per-gpu 4194304 $Q > $OUT/pmc6.log 2>&1 \
&& $P --pmc FETCH_SIZE -d $OUT/pmc_c3_fetch -o p --output-format csv -- python3 -u bench.py --workload C3 $Q > $OUT/pmc11.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_c3_write -o p --output-format csv -- python3 -u bench.py --workload C3 $Q > $OUT/pmc12.log 2>&1 \
&& step done
