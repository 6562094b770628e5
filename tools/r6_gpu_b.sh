# round-6 GPU session b: staged + shared-entries-under-churn tests, bench, A/B, diag, suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_sh.py tests/test_gpu_staged.py > $O/t1.log 2>&1 || { echo T1_FAIL; grep -E "FAIL|Error|assert" $O/t1.log | head -30; exit 1; }
tail -2 $O/t1.log
timeout -k 10 600 $PT tests/test_gpu_fullsize.py -k "class_coverage or c4_as" > $O/t2.log 2>&1 || { echo T2_FAIL; grep -E "FAIL|Error|assert" $O/t2.log | head -30; exit 1; }
tail -2 $O/t2.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python tools/r6_summ.py $O/bench.json
RAFTSTEP_SH=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --workload C4 --no-cpu-baseline > $O/c4_sh0.json 2> $O/c4_sh0.err && python tools/r6_summ.py $O/c4_sh0.json
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --workload C4 --no-cpu-baseline > $O/c4_sh1.json 2> $O/c4_sh1.err && python tools/r6_summ.py $O/c4_sh1.json
timeout -k 10 300 python -u tools/lean_diag.py --modes 0,256 --pipeline 1,0 > $O/lean_diag.log 2>&1; cat $O/lean_diag.log
timeout -k 10 1200 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ --ignore=tests/test_gpu_staged.py --ignore=tests/test_gpu_sh.py > $O/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/suite.log | head -30; exit 1; }
tail -2 $O/suite.log
