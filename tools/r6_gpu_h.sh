# round-6 GPU session h: dense isolation plane (whole suite) + list-kernel grid cap A/B on C4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
tail -1 $O/gpu_tests.log
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused --extra none"
for cap in 0 384 256 128 64; do
  RAFTSTEP_LIST_BLOCKS=$cap timeout -k 10 200 $B --workload C4 > $O/c4_cap$cap.json 2>/dev/null || exit 1
  echo "cap $cap"; python3 tools/r6_summ.py $O/c4_cap$cap.json
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c4_fetch -o p --output-format csv -- python3 -u bench.py --workload C4 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count > $O/pmc_c4_f.log 2>&1 || exit 1
echo PMC_OK
