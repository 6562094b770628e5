#!/bin/bash
# PMC summaries (profiles/pmc_*.json) from an evidence session's raw passes:
#   bash tools/pmc_all.sh gpurun_out/r4m
set -e
O=$1; C=$(git rev-parse --short HEAD)
B=$O/bench.json
W2=$(python3 -c "import json;print(json.load(open('$B'))['config']['workload'])")
W4=$(python3 -c "import json;print(json.load(open('$B'))['extra_workloads']['C4']['workload'])")
W5=$(python3 -c "import json;print(json.load(open('$B'))['extra_workloads']['C5']['workload'])")
W2X=$(python3 -c "import json;print(json.load(open('$B'))['extra_workloads']['C2X']['workload'])")
# algorithmic bytes per group-step (bench.py lean_bytes): the line's own, so
# that a change of storage form (shared entries: C2 52 B, C5 1064 B) follows
LB() { python3 -c "import json;d=json.load(open('$B'));x=d if '$1'=='C2' else d['extra_workloads']['$1'];print(int(x['roofline']['bytes_per_group_step']))"; }
S="python3 tools/pmc_summary.py --calib-fetch $O/pmc_calib_fetch --calib-write $O/pmc_calib_write --commit $C"
$S --fetch $O/pmc_c2_fetch --write $O/pmc_c2_write --kernel tick_lean_kernel --workload "$W2" \
   --algorithmic-bytes $(($(LB C2)*1048576/2)) --skip 5 --take 40 --launches-per-tick 2 --out profiles/pmc_C2_lean.json > /dev/null
$S --fetch $O/pmc_c2x_fetch --write $O/pmc_c2x_write --kernel tick_lean_kernel --workload "$W2X" \
   --algorithmic-bytes $(($(LB C2X)*16777216/2)) --skip 5 --take 40 --launches-per-tick 2 --out profiles/pmc_C2X_lean.json > /dev/null
$S --fetch $O/pmc_c4_fetch --write $O/pmc_c4_write --kernel tick_lean_kernel --workload "$W4" \
   --algorithmic-bytes $(($(LB C4)*4194304)) --skip 53 --take 20 --out profiles/pmc_C4_lean.json > /dev/null
$S --fetch $O/pmc_c4_fetch --write $O/pmc_c4_write --kernel tick_list_kernel --workload "$W4" \
   --skip 53 --take 20 --out profiles/pmc_C4_list.json > /dev/null
$S --fetch $O/pmc_c5_fetch --write $O/pmc_c5_write --kernel tick_lean_kernel --workload "$W5" \
   --algorithmic-bytes $(($(LB C5)*1048576/2)) --skip 5 --take 40 --launches-per-tick 2 --out profiles/pmc_C5_lean.json > /dev/null
# staged client values (round 6): the same kernels plus 8 E B per group-step
for w in C2S C4S; do
  [ -d "$O/pmc_${w,,}_fetch" ] || continue
  WW=$(python3 -c "import json;print(json.load(open('$B'))['extra_workloads']['$w']['workload'])")
  if [ $w = C2S ]; then
    $S --fetch $O/pmc_c2s_fetch --write $O/pmc_c2s_write --kernel tick_lean_kernel --workload "$WW" \
       --algorithmic-bytes $(($(LB C2S)*1048576/2)) --skip 5 --take 40 --launches-per-tick 2 --out profiles/pmc_C2S_lean.json > /dev/null
  else
    $S --fetch $O/pmc_c4s_fetch --write $O/pmc_c4s_write --kernel tick_lean_kernel --workload "$WW" \
       --algorithmic-bytes $(($(LB C4S)*4194304)) --skip 53 --take 20 --out profiles/pmc_C4S_lean.json > /dev/null
    $S --fetch $O/pmc_c4s_fetch --write $O/pmc_c4s_write --kernel tick_list_kernel --workload "$WW" \
       --skip 53 --take 20 --out profiles/pmc_C4S_list.json > /dev/null
  fi
done
# C5 with corrupted copies (rejections timed): one lean launch per tick (no split: the list runs)
if [ -d "$O/pmc_c5v_fetch" ]; then
  WW=$(python3 -c "import json;print(json.load(open('$B'))['extra_workloads']['C5V']['workload'])")
  $S --fetch $O/pmc_c5v_fetch --write $O/pmc_c5v_write --kernel tick_lean_kernel --workload "$WW" \
     --algorithmic-bytes $(($(LB C5V)*1048576)) --skip 5 --take 20 --out profiles/pmc_C5V_lean.json > /dev/null
  $S --fetch $O/pmc_c5v_fetch --write $O/pmc_c5v_write --kernel tick_list_kernel --workload "$WW" \
     --skip 5 --take 20 --out profiles/pmc_C5V_list.json > /dev/null
fi
for f in C2_lean C2X_lean C4_lean C4_list C5_lean C2S_lean C4S_lean C4S_list C5V_lean C5V_list; do
  [ -f profiles/pmc_$f.json ] || continue
  python3 -c "import json; d=json.load(open('profiles/pmc_$f.json')); print('$f', round(d.get('hbm_bytes_per_tick', d['hbm_bytes_per_launch'])/1e6,1), 'MB/tick', d.get('traffic_over_algorithmic'))"
done
