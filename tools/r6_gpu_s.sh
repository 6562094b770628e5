# round-6 GPU session s: C5V interleaved A/B — lean kernel's CRC check of corrupted copies (abcrc) vs pass-on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6s; mkdir -p $O
B="python3 -u bench.py --steps 20 --warmup 5 --no-fused --no-cpu-baseline --extra none"
for i in 1 2; do
  timeout -k 10 300 $B --workload C5V > $O/c5v_new_$i.json 2>/dev/null || exit 1
  echo new; python3 tools/r6_summ.py $O/c5v_new_$i.json | head -1
  RAFTSTEP_LIB=tools/bin/abcrc/libraftstep.so timeout -k 10 300 $B --workload C5V > $O/c5v_old_$i.json 2>/dev/null || exit 1
  echo old; python3 tools/r6_summ.py $O/c5v_old_$i.json | head -1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5v -o run --output-format csv -- python3 -u bench.py --workload C5V --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count > $O/prof.log 2>&1 || exit 1
echo PROF_OK
