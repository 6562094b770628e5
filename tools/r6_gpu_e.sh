# round-6 GPU session e: SH kept through rejections (REF + CRC), tests + C5V A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_sh.py tests/test_gpu_staged.py -k "corrupt or c5 or shared" > $O/t1.log 2>&1 || { echo T1_FAIL; grep -E "FAIL|Error|assert" $O/t1.log | head -30; exit 1; }
tail -2 $O/t1.log
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused"
timeout -k 10 200 $B --workload C5V > $O/c5v.json 2>/dev/null && python tools/r6_summ.py $O/c5v.json
RAFTSTEP_SH_KEEP=0 timeout -k 10 200 $B --workload C5V > $O/c5v_keep0.json 2>/dev/null && python tools/r6_summ.py $O/c5v_keep0.json
RAFTSTEP_SH=0 timeout -k 10 200 $B --workload C5V > $O/c5v_sh0.json 2>/dev/null && python tools/r6_summ.py $O/c5v_sh0.json
timeout -k 10 200 $B --workload C5 > $O/c5.json 2>/dev/null && python tools/r6_summ.py $O/c5.json
