# round-6 GPU session v: shared ring in 16-slot chunks for C5V (RAFTSTEP_SH_CHUNK) — tests, interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6v; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_sh.py tests/test_gpu_staged.py tests/test_gpu_fullsize.py -k "lagging or corrupt or c5 or C5" > $O/t0.log 2>&1 || { echo T0_FAIL; grep -E "FAIL|Error|assert" $O/t0.log | head; exit 1; }
tail -1 $O/t0.log
B="python3 -u bench.py --steps 20 --warmup 5 --no-fused --no-cpu-baseline --extra none"
for i in 1 2; do for c in 1 0; do
  RAFTSTEP_SH_CHUNK=$c timeout -k 10 300 $B --workload C5V > $O/c5v_ch${c}_$i.json 2>/dev/null || exit 1
  echo "chunk $c"; python3 tools/r6_summ.py $O/c5v_ch${c}_$i.json | head -1
done; done
timeout -k 10 300 $B --workload C5 > $O/c5.json 2>/dev/null || exit 1
python3 tools/r6_summ.py $O/c5.json | head -1
