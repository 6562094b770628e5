set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
OUTDIR=mr1/ab VARIANTS="base minreg" ARGS="--workload C4" ROUNDS=4 bash tools/gpu_ab.sh && \
OUTDIR=mr1/abr VARIANTS="base minreg" ARGS="--workload C4R" ROUNDS=2 bash tools/gpu_ab.sh && \
OUTDIR=mr1/ab2 VARIANTS="base minreg" ARGS="" ROUNDS=3 bash tools/gpu_ab.sh
