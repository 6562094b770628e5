#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUTDIR:-r3bis}
mkdir -p $OUT
for v in "RAFTSTEP_SLOW_EVERY=3 RAFTSTEP_PIPELINE=1" "RAFTSTEP_SLOW_EVERY=3 RAFTSTEP_PIPELINE=0" "RAFTSTEP_SLOW_EVERY=3 RAFTSTEP_PIPELINE=1 RAFTSTEP_OVERLAP_GENERAL=0" "RAFTSTEP_SLOW_EVERY=1 RAFTSTEP_PIPELINE=1"; do
  echo "== $v" >> $OUT/bisect.log
  env $v timeout -k 10 300 python -u tools/r3/bisect_dist.py 3 >> $OUT/bisect.log 2>&1 || exit 1
done
