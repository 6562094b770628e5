#!/bin/bash
# The per-call pipeline choice (RAFTSTEP_PIPELINE=2): the pipeline tests, then
# C4 and C4R with the pipeline off / on / auto (each call's choice and the
# previous call's last list size on stderr), then the whole GPU suite and the
# driver's bench command for the committed defaults.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3auto}
mkdir -p $OUT
B="python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --repeats 3"
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread > $OUT/pipe_tests.log 2>&1 || exit 1
for w in C4R C4; do
  for m in 0 1 2; do
    echo "== $(date +%T) $w $m" >> $OUT/progress.log
    RAFTSTEP_PIPELINE=$m RAFTSTEP_DEBUG_PIPE=1 timeout -k 10 300 $B --workload $w > $OUT/${w}_p$m.json 2> $OUT/${w}_p$m.err || exit 1
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
&& timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --groups-per-gpu 4194304 --no-cpu-baseline > $OUT/bench_c2_4m.json 2> $OUT/bench_c2_4m.err \
&& timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --repeats 2 --no-cpu-baseline > $OUT/prof_c2.log 2>&1
