# round-6 GPU session p: list kernel active lanes per wave (RAFTSTEP_LIST_LANES builds) A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6p; mkdir -p $O
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused --extra none --no-list-count"
run() {  # variant workload tag
  if [ "$1" = 64 ]; then L=; else L=tools/bin/ll$1/libraftstep.so; fi
  RAFTSTEP_LIB=$L timeout -k 10 200 $B --workload $2 > $O/$2_ll$1_$3.json 2>/dev/null || exit 1
  echo "$2 lanes $1"; python3 tools/r6_summ.py $O/$2_ll$1_$3.json | head -1
}
for i in 1 2; do for v in 64 32 16; do run $v C4 $i; done; done
for w in C4S C4R; do for v in 64 32 16; do run $v $w 1; done; done
