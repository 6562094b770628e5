#!/bin/bash
# GPU parity suite only (each run bounded; stops at the first failure).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:-} > gpurun_out/gpu_tests.log 2>&1
