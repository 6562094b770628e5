set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
OUTDIR=r4o bash tools/gpu_session.sh tests smoke bench && bash tools/r4/n2.sh
