# round-6 GPU session n: pipeline depth 3 (RAFTSTEP_PIPELINE_DEPTH) tests, then C4-family A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py -k depth3 > $O/t1.log 2>&1 \
  || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/t1.log | head -30; exit 1; }
tail -1 $O/t1.log
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused --extra none --no-list-count"
for i in 1 2; do
  for d in 3 2; do
    RAFTSTEP_PIPELINE_DEPTH=$d timeout -k 10 200 $B --workload C4 > $O/c4_d${d}_$i.json 2>/dev/null || exit 1
    echo "C4 depth $d"; python3 tools/r6_summ.py $O/c4_d${d}_$i.json | head -1
  done
done
for w in C4S C4R C4REF; do for d in 3 2; do
  RAFTSTEP_PIPELINE_DEPTH=$d timeout -k 10 200 $B --workload $w > $O/${w}_d${d}.json 2>/dev/null || exit 1
  echo "$w depth $d"; python3 tools/r6_summ.py $O/${w}_d${d}.json | head -1
done; done
