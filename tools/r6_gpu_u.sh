# round-6 GPU session u: wave-cooperative list-kernel batch writes — C5V A/B first, then the whole suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6u; mkdir -p $O
B="python3 -u bench.py --steps 20 --warmup 5 --no-fused --no-cpu-baseline --extra none"
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_sh.py tests/test_gpu_staged.py -k "lagging or corrupt or c5" > $O/t0.log 2>&1 || { echo T0_FAIL; grep -E "FAIL|Error|assert" $O/t0.log | head; exit 1; }
tail -1 $O/t0.log
for w in C5V C5 C4; do
  timeout -k 10 300 $B --workload $w > $O/$w.json 2>/dev/null || exit 1
  python3 tools/r6_summ.py $O/$w.json | head -1
done
RAFTSTEP_LIB=tools/bin/wprof/libraftstep.so timeout -k 10 240 python3 -u tools/list_prof.py --workload C5V > $O/list_prof_c5v.log 2>&1 || exit 1
grep -A8 per_step_cycles $O/list_prof_c5v.log; grep list_kernel_us $O/list_prof_c5v.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
tail -1 $O/gpu_tests.log
