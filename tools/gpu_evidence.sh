#!/bin/bash
# Round evidence in one GPU session: parity suite, the bench lines of C2
# (headline, with cpu_baseline), C2 at 4M groups, C4 and C5, a
# rocprofv3 --kernel-trace --stats summary of each, and the FETCH_SIZE /
# WRITE_SIZE passes (separate runs, calibrated by tools/pmc_calib) of C2 and
# C4. Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/ev
mkdir -p $OUT
P="timeout -s KILL 120 rocprofv3"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& timeout -k 10 240 python -u bench.py > $OUT/bench_c2.log 2>&1 \
&& timeout -k 10 240 python -u bench.py --groups-per-gpu 4194304 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_c2_4m.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --workload C4 --steps 100 --warmup 16 > $OUT/bench_c4.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --workload C5 --steps 100 --warmup 5 > $OUT/bench_c5.log 2>&1 \
&& timeout -k 10 180 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c2 -o run --output-format csv -- python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/prof_c2.log 2>&1 \
&& timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c4 -o run --output-format csv -- python3 -u bench.py --workload C4 --steps 100 --warmup 16 --no-cpu-baseline > $OUT/prof_c4.log 2>&1 \
&& timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c5 -o run --output-format csv -- python3 -u bench.py --workload C5 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/prof_c5.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_calib_fetch -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc1.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_calib_write -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc2.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_c2_fetch -o p --output-format csv -- python3 -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/pmc3.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c2_write -o p --output-format csv -- python3 -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/pmc4.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_c4_fetch -o p --output-format csv -- python3 -u bench.py --workload C4 --steps 24 --warmup 2 --no-cpu-baseline > $OUT/pmc5.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c4_write -o p --output-format csv -- python3 -u bench.py --workload C4 --steps 24 --warmup 2 --no-cpu-baseline > $OUT/pmc6.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_c5_fetch -o p --output-format csv -- python3 -u bench.py --workload C5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/pmc7.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c5_write -o p --output-format csv -- python3 -u bench.py --workload C5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/pmc8.log 2>&1
