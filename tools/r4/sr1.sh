set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/sr1 && mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
OUTDIR=sr1/ab VARIANTS="prev base" ARGS="" ROUNDS=4 bash tools/gpu_ab.sh && \
OUTDIR=sr1/ab5 VARIANTS="prev base" ARGS="--workload C5" ROUNDS=2 bash tools/gpu_ab.sh
