set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
OUTDIR=og1/ab VARIANTS="og1+RAFTSTEP_OVERLAP_GENERAL=1 base og3+RAFTSTEP_OVERLAP_GENERAL=3" ARGS="--workload C4" ROUNDS=3 bash tools/gpu_ab.sh && \
OUTDIR=og1/abr VARIANTS="og1+RAFTSTEP_OVERLAP_GENERAL=1 base og3+RAFTSTEP_OVERLAP_GENERAL=3" ARGS="--workload C4R" ROUNDS=2 bash tools/gpu_ab.sh
