set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
OUTDIR=lg1/ab VARIANTS="base lg3 lg4 lg6" ARGS="--workload C4" ROUNDS=2 bash tools/gpu_ab.sh && \
OUTDIR=lg1/abr VARIANTS="base lg4" ARGS="--workload C4R" ROUNDS=1 bash tools/gpu_ab.sh && \
OUTDIR=lg1/ab2 VARIANTS="base lg4" ARGS="" ROUNDS=2 bash tools/gpu_ab.sh
