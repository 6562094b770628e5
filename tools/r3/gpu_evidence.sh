#!/bin/bash
# Round-3 evidence in one GPU session: every bench line at the driver's
# protocol (--steps 20 --warmup 5; C2 with cpu_baseline), rocprofv3
# kernel-trace summaries of C2 and C4, FETCH_SIZE / WRITE_SIZE passes
# (separate runs, calibrated by tools/pmc_calib) of C2, C2 at 2^22, C3, C4
# and C5, and the 2-rank same-GPU rehearsal of the N>1 bench path. Every
# GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3ev}
mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 5"
P="timeout -s KILL 120 rocprofv3"
Q="--steps 20 --warmup 5 --repeats 1 --no-cpu-baseline"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step c2 && timeout -k 10 300 $B > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
&& step c2_4m && timeout -k 10 300 $B --groups-per-gpu 4194304 --no-cpu-baseline > $OUT/bench_c2_4m.json 2> $OUT/bench_c2_4m.err \
&& step c3 && timeout -k 10 300 $B --workload C3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err \
&& step c4 && timeout -k 10 300 $B --workload C4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err \
&& step c4r && timeout -k 10 300 $B --workload C4R --no-cpu-baseline > $OUT/bench_c4r.json 2> $OUT/bench_c4r.err \
&& step c4ref && timeout -k 10 300 $B --workload C4REF --no-cpu-baseline > $OUT/bench_c4ref.json 2> $OUT/bench_c4ref.err \
&& step c5 && timeout -k 10 300 $B --workload C5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err \
&& step prof_c2 && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 -u bench.py $Q > $OUT/prof_c2.log 2>&1 \
&& step prof_c4 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- python3 -u bench.py --workload C4 $Q > $OUT/prof_c4.log 2>&1 \
&& step pmc && $P --pmc FETCH_SIZE -d $OUT/pmc_calib_fetch -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc1.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_calib_write -o p --output-format csv -- ./tools/pmc_calib > $OUT/pmc2.log 2>&1 \
&& $P --pmc FETCH_SIZE -d $OUT/pmc_c2_fetch -o p --output-format csv -- python3 -u bench.py $Q > $OUT/pmc3.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_c2_write -o p --output-format csv -- python3 -u bench.py $Q > $OUT/pmc4.log 2>&1 \
&& $P --pmc FETCH_SIZE -d $OUT/pmc_c2_4m_fetch -o p --output-format csv -- python3 -u bench.py --groups-per-gpu 4194304 $Q > $OUT/pmc5.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_c2_4m_write -o p --output-format csv -- python3 -u bench.py --groups-per-gpu 4194304 $Q > $OUT/pmc6.log 2>&1 \
&& $P --pmc FETCH_SIZE -d $OUT/pmc_c4_fetch -o p --output-format csv -- python3 -u bench.py --workload C4 $Q > $OUT/pmc7.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_c4_write -o p --output-format csv -- python3 -u bench.py --workload C4 $Q > $OUT/pmc8.log 2>&1 \
&& $P --pmc FETCH_SIZE -d $OUT/pmc_c5_fetch -o p --output-format csv -- python3 -u bench.py --workload C5 --steps 10 --warmup 2 --repeats 1 --no-cpu-baseline > $OUT/pmc9.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_c5_write -o p --output-format csv -- python3 -u bench.py --workload C5 --steps 10 --warmup 2 --repeats 1 --no-cpu-baseline > $OUT/pmc10.log 2>&1 \
&& $P --pmc FETCH_SIZE -d $OUT/pmc_c3_fetch -o p --output-format csv -- python3 -u bench.py --workload C3 $Q > $OUT/pmc11.log 2>&1 \
&& $P --pmc WRITE_SIZE -d $OUT/pmc_c3_write -o p --output-format csv -- python3 -u bench.py --workload C3 $Q > $OUT/pmc12.log 2>&1 \
&& step rehearsal && RAFTSTEP_BENCH_SAME_DEVICE=1 timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --groups-per-gpu 262144 > $OUT/bench_2rank.log 2>&1 \
&& step done
