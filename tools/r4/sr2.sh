set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/sr2 && mkdir -p $O
for r in 1 2; do
RAFTSTEP_LIB=ablib/prev/libraftstep.so timeout -k 10 300 python3 -u tools/overhead_probe.py > $O/prev_$r.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/overhead_probe.py > $O/base_$r.txt 2>&1 || exit 1
done
