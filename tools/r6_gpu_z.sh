# round-6 GPU session z: general-kernel overlap depth 4 / 5 — pipeline tests, C4-family A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6z; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py -k "-4- or -5-" > $O/t0.log 2>&1 || { echo T0_FAIL; grep -E "FAIL|Error|assert" $O/t0.log | head; exit 1; }
tail -1 $O/t0.log
B="python3 -u bench.py --steps 20 --warmup 5 --no-fused --no-cpu-baseline --extra none --no-list-count"
for i in 1 2; do for d in 3 4 5; do
  RAFTSTEP_OVERLAP_GENERAL=$d timeout -k 10 300 $B --workload C4 > $O/c4_d${d}_$i.json 2>/dev/null || exit 1
  echo "C4 overlap $d"; python3 tools/r6_summ.py $O/c4_d${d}_$i.json | head -1
done; done
for w in C4S C4R C4REF; do for d in 3 5; do
  RAFTSTEP_OVERLAP_GENERAL=$d timeout -k 10 300 $B --workload $w > $O/${w}_d${d}.json 2>/dev/null || exit 1
  echo "$w overlap $d"; python3 tools/r6_summ.py $O/${w}_d${d}.json | head -1
done; done
