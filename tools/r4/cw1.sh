set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/cw1 && mkdir -p $O
for r in 1 2; do
PROBE_COMM=1 RAFTSTEP_COMM_WINDOW_FLUSH=1 timeout -k 10 300 python3 -u tools/overhead_probe.py > $O/win_$r.txt 2>&1 && \
PROBE_COMM=1 timeout -k 10 300 python3 -u tools/overhead_probe.py > $O/end_$r.txt 2>&1 || exit 1
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > $O/dist.log 2>&1
