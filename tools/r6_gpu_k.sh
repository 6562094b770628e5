# round-6 GPU session k: list kernel slots sorted by form (RAFTSTEP_LIST_SORT) A/B, then the whole suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused --extra none --no-list-count"
for i in 1 2; do
  for ls in 1 0; do
    RAFTSTEP_LIST_SORT=$ls timeout -k 10 200 $B --workload C4 > $O/c4_ls${ls}_$i.json 2>/dev/null || exit 1
    echo "C4 sort $ls"; python3 tools/r6_summ.py $O/c4_ls${ls}_$i.json | head -1
  done
done
for w in C4S C4R; do for ls in 1 0; do
  RAFTSTEP_LIST_SORT=$ls timeout -k 10 200 $B --workload $w > $O/${w}_ls${ls}.json 2>/dev/null || exit 1
  echo "$w sort $ls"; python3 tools/r6_summ.py $O/${w}_ls${ls}.json | head -1
done; done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
tail -1 $O/gpu_tests.log
