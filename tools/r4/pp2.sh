set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/pp2 && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
OUTDIR=pp2/ab VARIANTS="evk0+RAFTSTEP_PP_EVK=0 base" ARGS="--workload C4" ROUNDS=3 bash tools/gpu_ab.sh && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c4 -o run --output-format csv -- python3 -u bench.py --workload C4 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count > $O/c4.log 2>&1
