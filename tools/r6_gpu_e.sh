# round-6 GPU session e: C5V with / without shared entries (lagging-follower class on)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e; mkdir -p $O
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused"
RAFTSTEP_SH=0 timeout -k 10 200 $B --workload C5V > $O/c5v_sh0.json 2>/dev/null && python tools/r6_summ.py $O/c5v_sh0.json
RAFTSTEP_SH=0 timeout -k 10 200 $B --workload C5 > $O/c5_sh0.json 2>/dev/null && python tools/r6_summ.py $O/c5_sh0.json
timeout -k 10 200 $B --workload C5V > $O/c5v.json 2>/dev/null && python tools/r6_summ.py $O/c5v.json
