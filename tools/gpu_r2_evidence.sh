#!/bin/bash
# Round 2 evidence (two-pass tick) in one GPU session: the GPU test suite, every bench line
# (C2 headline with cpu_baseline, C2 at 4M groups, C3 on one GPU, C4 at
# general-kernel cadence 8 and 1, C4R, C4REF, C5), rocprofv3 kernel-trace
# summaries of C2 and C4, FETCH_SIZE / WRITE_SIZE passes (separate runs,
# calibrated by tools/pmc_calib) of C2, C2-4M and C4, and the 2-rank
# same-GPU rehearsal of the N>1 bench path. Every GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2ev2}
mkdir -p $OUT
B="python3 -u bench.py"
P="timeout -s KILL 120 rocprofv3"
C4A="--workload C4 --steps 24 --warmup 200 --repeats 1 --no-cpu-baseline"
C5A="--workload C5 --steps 10 --warmup 2 --repeats 1 --no-cpu-baseline"
C3A="--workload C3 --steps 20 --warmup 2 --repeats 1 --no-cpu-baseline"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step tests && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& step c2 && timeout -k 10 300 $B > $OUT/bench_c2.log 2>&1 \
&& step c2_4m && timeout -k 10 300 $B --groups-per-gpu 4194304 --steps 100 --no-cpu-baseline > $OUT/bench_c2_4m.log 2>&1 \
&& step c3 && timeout -k 10 300 $B --workload C3 --no-cpu-baseline > $OUT/bench_c3.log 2>&1 \
&& step c4 && RAFTSTEP_SLOW_EVERY=8 timeout -k 10 300 $B --workload C4 --steps 100 --warmup 200 > $OUT/bench_c4.log 2>&1 \
&& step c4_se1 && RAFTSTEP_SLOW_EVERY=1 timeout -k 10 300 $B --workload C4 --steps 100 --warmup 200 --no-cpu-baseline > $OUT/bench_c4_se1.log 2>&1 \
&& step c4r && timeout -k 10 300 $B --workload C4R --steps 100 --warmup 200 --no-cpu-baseline > $OUT/bench_c4r.log 2>&1 \
&& step c4ref && timeout -k 10 300 $B --workload C4REF --steps 64 --warmup 16 --no-cpu-baseline > $OUT/bench_c4ref.log 2>&1 \
&& step c5 && timeout -k 10 300 $B --workload C5 --steps 50 --warmup 5 > $OUT/bench_c5.log 2>&1 \
&& step prof_c2 && timeout -k 10 180 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c2 -o run --output-format csv -- python3 -u bench.py --steps 200 --warmup 20 --repeats 1 --no-cpu-baseline > $OUT/prof_c2.log 2>&1 \
&& step prof_c4 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c4 -o run --output-format csv -- python3 -u bench.py --workload C4 --steps 64 --warmup 200 --repeats 1 --no-cpu-baseline > $OUT/prof_c4.log 2>&1 \
&& step pmc && $P --pmc FETCH_SIZE -T -d $OUT/pmc_calib_fetch -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc1.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_calib_write -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc2.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_c2_fetch -o p --output-format csv -- python3 -u bench.py --steps 20 --warmup 2 --repeats 1 --no-cpu-baseline > $OUT/pmc3.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c2_write -o p --output-format csv -- python3 -u bench.py --steps 20 --warmup 2 --repeats 1 --no-cpu-baseline > $OUT/pmc4.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_c2_4m_fetch -o p --output-format csv -- python3 -u bench.py --groups-per-gpu 4194304 --steps 20 --warmup 2 --repeats 1 --no-cpu-baseline > $OUT/pmc5.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c2_4m_write -o p --output-format csv -- python3 -u bench.py --groups-per-gpu 4194304 --steps 20 --warmup 2 --repeats 1 --no-cpu-baseline > $OUT/pmc6.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_c4_fetch -o p --output-format csv -- python3 -u bench.py $C4A > $OUT/pmc7.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c4_write -o p --output-format csv -- python3 -u bench.py $C4A > $OUT/pmc8.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_c5_fetch -o p --output-format csv -- python3 -u bench.py $C5A > $OUT/pmc9.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c5_write -o p --output-format csv -- python3 -u bench.py $C5A > $OUT/pmc10.log 2>&1 \
&& $P --pmc FETCH_SIZE -T -d $OUT/pmc_c3_fetch -o p --output-format csv -- python3 -u bench.py $C3A > $OUT/pmc11.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_c3_write -o p --output-format csv -- python3 -u bench.py $C3A > $OUT/pmc12.log 2>&1 \
&& step rehearsal && RAFTSTEP_BENCH_SAME_DEVICE=1 timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 30 --warmup 3 --groups-per-gpu 262144 > $OUT/bench_2rank.log 2>&1 \
&& step done
