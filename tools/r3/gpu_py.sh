#!/bin/bash
# run one python diagnostic under a time limit, output to gpurun_out/$OUTDIR/py.log
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/${OUTDIR:-r3py}
timeout -k 10 ${LIMIT:-600} python -u "$@" > gpurun_out/${OUTDIR:-r3py}/py.log 2>&1
