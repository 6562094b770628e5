# round-6 GPU session d: staged moves / returns, REF lagging-follower catch-up, SH under churn A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6d; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_staged.py tests/test_gpu_sh.py > $O/t1.log 2>&1 || { echo T1_FAIL; grep -E "FAIL|Error|assert" $O/t1.log | head -30; exit 1; }
tail -2 $O/t1.log
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused"
for i in 1 2; do
  timeout -k 10 200 $B --workload C4 > $O/c4_$i.json 2>/dev/null && python tools/r6_summ.py $O/c4_$i.json
  RAFTSTEP_SH=2 timeout -k 10 200 $B --workload C4 > $O/c4sh2_$i.json 2>/dev/null && python tools/r6_summ.py $O/c4sh2_$i.json
done
RAFTSTEP_VX=0 timeout -k 10 200 $B --workload C4 > $O/c4vx0.json 2>/dev/null && python tools/r6_summ.py $O/c4vx0.json
timeout -k 10 200 $B --workload C4S > $O/c4s.json 2>/dev/null && python tools/r6_summ.py $O/c4s.json
timeout -k 10 200 $B --workload C5V > $O/c5v.json 2>/dev/null && python tools/r6_summ.py $O/c5v.json
timeout -k 10 1200 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ --ignore=tests/test_gpu_staged.py --ignore=tests/test_gpu_sh.py > $O/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/suite.log | head -30; exit 1; }
tail -2 $O/suite.log
