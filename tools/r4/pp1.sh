set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/pp1 && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_engine_checks.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
OUTDIR=pp1/ab VARIANTS="pp0+RAFTSTEP_PINGPONG=0 base" ARGS="--workload C4" ROUNDS=3 bash tools/gpu_ab.sh && \
OUTDIR=pp1/abr VARIANTS="pp0+RAFTSTEP_PINGPONG=0 base" ARGS="--workload C4R" ROUNDS=2 bash tools/gpu_ab.sh && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c4 -o run --output-format csv -- python3 -u bench.py --workload C4 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count > $O/c4.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread > $O/fullsize.log 2>&1
