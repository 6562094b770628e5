#!/bin/bash
# summary of a tools/gpu_r3.sh run directory
d=gpurun_out/$1
grep -E "FAIL|passed|failed|Error" $d/gpu_tests.log 2>/dev/null | tail -10
grep "class counters" $d/gpu_tests.log 2>/dev/null | cut -c1-1600
for f in $d/bench_*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
r=d['roofline']
print('$f'.split('/')[-1], '%.4g'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'lean %.1f list %s region %.1f'%(r['avg_kernel_us'], r['list_kernel_us'], r['avg_region_us_per_tick']), 'frac %.3f'%r['frac'], d['stats_check'], [round(x,4) for x in d['timing']['repeat_ms_per_step']])
" 2>/dev/null; done
