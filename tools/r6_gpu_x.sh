# round-6 GPU session x: shard chunks (RAFTSTEP_SHARD_SB) — C4-family A/B, then the whole suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6x; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py -k "True-1" > $O/t0.log 2>&1 || { echo T0_FAIL; grep -E "FAIL|Error|assert" $O/t0.log | head; exit 1; }
tail -1 $O/t0.log
B="python3 -u bench.py --steps 20 --warmup 5 --no-fused --no-cpu-baseline --extra none --no-list-count"
for i in 1 2; do for sb in 6 0; do
  RAFTSTEP_SHARD_SB=$sb timeout -k 10 300 $B --workload C4 > $O/c4_sb${sb}_$i.json 2>/dev/null || exit 1
  echo "C4 sb $sb"; python3 tools/r6_summ.py $O/c4_sb${sb}_$i.json | head -1
done; done
for w in C4S C4R C5V; do for sb in 6 0; do
  RAFTSTEP_SHARD_SB=$sb timeout -k 10 300 $B --workload $w > $O/${w}_sb${sb}.json 2>/dev/null || exit 1
  echo "$w sb $sb"; python3 tools/r6_summ.py $O/${w}_sb${sb}.json | head -1
done; done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
tail -1 $O/gpu_tests.log
