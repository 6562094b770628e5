set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
OUTDIR=la1/ab VARIANTS="base la32 la16 lp0" ARGS="--workload C4" ROUNDS=3 bash tools/gpu_ab.sh && \
OUTDIR=la1/abr VARIANTS="base la32 lp0" ARGS="--workload C4R" ROUNDS=1 bash tools/gpu_ab.sh
