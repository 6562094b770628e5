#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/${OUTDIR:-r3p}
timeout -k 10 600 python -u tools/r3/fault_probe.py "$@" > gpurun_out/${OUTDIR:-r3p}/probe.log 2>&1
