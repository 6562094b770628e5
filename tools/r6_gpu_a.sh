set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_staged.py > $O/staged.log 2>&1 || { echo STAGED_FAIL; tail -30 $O/staged.log; exit 1; }
tail -3 $O/staged.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload C2S --no-fused --extra C4S,C5V,C4 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.log; exit 1; }
python - <<'P'
import json
d=json.loads(open("gpurun_out/r6a/bench.log").read().strip().splitlines()[-1])
print("C2S", d["value"], d["roofline"]["frac"], d["roofline"]["avg_kernel_us_per_tick"], d.get("stats_check"))
for k,x in d.get("extra_workloads",{}).items():
    print(k, x.get("value"), x.get("roofline",{}).get("frac"), x.get("roofline",{}).get("avg_kernel_us_per_tick"), x.get("stats_check"), x.get("pcie_inclusive",{}).get("value"), x.get("verification"))
P
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ --ignore=tests/test_gpu_staged.py > $O/suite.log 2>&1 || { echo SUITE_FAIL; tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
