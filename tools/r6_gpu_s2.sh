# round-6 GPU session s2: C2 / C2X split steady tick on / off, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6s2; mkdir -p $O
B="python3 -u bench.py --steps 20 --warmup 5 --no-fused --no-cpu-baseline --extra none"
for i in 1 2; do for sp in 1 0; do
  RAFTSTEP_SPLIT_STEADY=$sp timeout -k 10 300 $B > $O/c2_sp${sp}_$i.json 2>/dev/null || exit 1
  echo "C2 split $sp"; python3 tools/r6_summ.py $O/c2_sp${sp}_$i.json | head -1
  RAFTSTEP_SPLIT_STEADY=$sp timeout -k 10 300 $B --workload C2X > $O/c2x_sp${sp}_$i.json 2>/dev/null || exit 1
  echo "C2X split $sp"; python3 tools/r6_summ.py $O/c2x_sp${sp}_$i.json | head -1
done; done
