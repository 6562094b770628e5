# round-6 GPU session r: several lagging followers on the fast path (C5V) — tests, C5V / C5 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_sh.py tests/test_gpu_staged.py tests/test_gpu_fullsize.py -k "lagging or corrupt or c5 or C5" > $O/t1.log 2>&1 \
  || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/t1.log | head -30; exit 1; }
tail -1 $O/t1.log; grep "class counters" $O/t1.log | head -3
B="python3 -u bench.py --steps 20 --warmup 5 --no-fused --extra none"
timeout -k 10 300 $B --workload C5V > $O/c5v.json 2>/dev/null || exit 1
python3 tools/r6_summ.py $O/c5v.json
RAFTSTEP_DEBUG_WORK=1 timeout -k 10 300 python3 -u tools/classes.py --workload C5V --ticks 20 > $O/classes_c5v.log 2>&1 || exit 1
head -8 $O/classes_c5v.log
timeout -k 10 300 $B --workload C5 > $O/c5.json 2>/dev/null || exit 1
python3 tools/r6_summ.py $O/c5.json
