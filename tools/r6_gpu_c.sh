# round-6 GPU session c: SH (coop copy-back) + staged (gather returns) tests, bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 700 $PT tests/test_gpu_sh.py tests/test_gpu_staged.py tests/test_gpu_multiproc.py > $O/t1.log 2>&1 || { echo T1_FAIL; grep -E "FAIL|Error|assert" $O/t1.log | head -30; exit 1; }
tail -2 $O/t1.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python tools/r6_summ.py $O/bench.json
RAFTSTEP_SH=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --workload C5V --no-cpu-baseline --no-fused > $O/c5v_sh0.json 2> $O/c5v_sh0.err && python tools/r6_summ.py $O/c5v_sh0.json
