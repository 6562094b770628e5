# round-6 GPU session i: C4 stream form A/B (ping-pong vs lean-stream/list-stream), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused --extra none --no-list-count"
for i in 1 2; do
  for pp in 1 0; do
    RAFTSTEP_PINGPONG=$pp timeout -k 10 200 $B --workload C4 > $O/c4_pp${pp}_$i.json 2>/dev/null || exit 1
    echo "pingpong $pp"; python3 tools/r6_summ.py $O/c4_pp${pp}_$i.json | head -1
  done
done
for pp in 1 0; do
  RAFTSTEP_PINGPONG=$pp timeout -k 10 200 $B --workload C4S > $O/c4s_pp${pp}.json 2>/dev/null || exit 1
  echo "C4S pingpong $pp"; python3 tools/r6_summ.py $O/c4s_pp${pp}.json | head -1
done
RAFTSTEP_PINGPONG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4_pp0 -o run --output-format csv -- python3 -u bench.py --workload C4 --steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count > $O/prof_pp0.log 2>&1 || exit 1
echo PROF_OK
