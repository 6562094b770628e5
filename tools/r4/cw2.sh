set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/cw2 && mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_c3.py -x -q --timeout 120 --timeout-method thread > $O/dist.log 2>&1 && \
for r in 1 2; do PROBE_COMM=1 timeout -k 10 300 python3 -u tools/overhead_probe.py > $O/probe_$r.txt 2>&1 || exit 1; done
