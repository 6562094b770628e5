#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c5 -o run --output-format csv -- python3 -u bench.py --workload C5 --steps 40 --warmup 3 --no-cpu-baseline > $OUT/prof_c5.log 2>&1 \
&& timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -T -d $OUT/pmc_c5 -o p --output-format csv -- python3 -u bench.py --workload C5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/pmc_c5.log 2>&1 \
&& RAFTSTEP_BENCH_SAME_DEVICE=1 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 30 --warmup 3 --groups-per-gpu 262144 > $OUT/bench_2rank.log 2>&1
