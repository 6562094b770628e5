set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/pp3 && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine_checks.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
OUTDIR=pp3/ab VARIANTS="evk0+RAFTSTEP_PP_EVK=0 base" ARGS="" ROUNDS=4 bash tools/gpu_ab.sh && \
OUTDIR=pp3/ab5 VARIANTS="evk0+RAFTSTEP_PP_EVK=0 base" ARGS="--workload C5" ROUNDS=2 bash tools/gpu_ab.sh
