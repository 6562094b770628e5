# round-6 GPU session tr: per-tick client-entry constants from the host (Trace n_tick / eb_tick) — interleaved A/B + SQ
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6tr; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_engine_checks.py -k "True-1 or fused or split" > $O/t0.log 2>&1 || { echo T0_FAIL; grep -E "FAIL|Error|assert" $O/t0.log | head; exit 1; }
tail -1 $O/t0.log
B="python3 -u bench.py --steps 20 --warmup 5 --no-fused --no-cpu-baseline --extra none --no-list-count"
for i in 1 2; do for v in new old; do
  if [ $v = old ]; then L=tools/bin/abtr/libraftstep.so; else L=; fi
  for w in C2 C2X C4 C5; do
    RAFTSTEP_LIB=$L timeout -k 10 300 $B --workload $w > $O/${w}_${v}_$i.json 2>/dev/null || exit 1
    echo "$w $v"; python3 tools/r6_summ.py $O/${w}_${v}_$i.json | head -1
  done
done; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d $O/sq_c2 -o p --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count > $O/sq.log 2>&1 || exit 1
python3 tools/sq_summary.py $O/sq_c2
