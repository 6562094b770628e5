#!/bin/bash
# one line per bench log: value, ms/tick, steady-state kernel us, list kernel us, frac
for f in "$@"; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('%-40s %.3e  %.4f ms  k %.1f us  list %s  frac %.2f' % ('$f'.split('/')[-1], d['value'], d['ms_per_step'], r.get('avg_kernel_us'), r.get('list_kernel_us'), r.get('frac')))" 2>/dev/null || echo "$f: no result"; done
