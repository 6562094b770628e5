# round-6 GPU session l: list kernel reads giso only under an active window; leader-isolation tests, C4 bench + list PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_pipeline.py tests/test_gpu_raft.py tests/test_gpu_vx.py tests/test_gpu_staged.py > $O/t1.log 2>&1 \
  || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/t1.log | head -30; exit 1; }
tail -1 $O/t1.log
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused --extra none"
timeout -k 10 200 $B --workload C4 > $O/c4.json 2>/dev/null || exit 1
python3 tools/r6_summ.py $O/c4.json | head -1
Q="--steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c4_fetch -o p --output-format csv -- python3 -u bench.py --workload C4 $Q > $O/pmc_f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c4_write -o p --output-format csv -- python3 -u bench.py --workload C4 $Q > $O/pmc_w.log 2>&1 || exit 1
echo PMC_OK
