#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/${OUTDIR:-r3d}
timeout -k 10 600 python -u tools/r3/${DBG:-debug_block}.py "$@" > gpurun_out/${OUTDIR:-r3d}/dbg.log 2>&1
