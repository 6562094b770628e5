#!/bin/bash
# One GPU session (run through gpurun from the repo root): the steps named on
# the command line, in order, each under its own time limit; the first
# failure ends the session. Output under gpurun_out/$OUTDIR.
#   tests     the whole -m gpu suite
#   bench     bench.py with the driver's protocol (--steps 20 --warmup 5): the
#             C2 headline + fused block + C4 / C5 extra workloads
#   prof      rocprofv3 --kernel-trace --stats of the C2 headline line (same
#             protocol, one repeat; the lean kernel's mean duration)
#   profc4    the same for C4 (lean + list kernels)
#   pmc       FETCH_SIZE / WRITE_SIZE passes (separate runs) of the calibration
#             kernel and of the C2 headline (tools/pmc_summary.py)
#   pmcc4     the same for C4 (lean and list kernels)
#   profc2x / pmcc2x  kernel trace / PMC passes of C2X (C2 at 2^24 groups, L3-proof)
#   sqc5      one SQ counter pass of C5 (LDS instructions and waits, busy cycles)
#   smoke     __graft_entry__.smoke()
#   bench:ARGS  bench.py with extra arguments (ARGS: comma-separated)
#   prof:W / pmc:W  kernel trace / PMC passes of bench.py --workload W (e.g. C2S, C4S)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
# LIB=path: run every step with that build of libraftstep.so (A/B evidence)
[ -n "$LIB" ] && export RAFTSTEP_LIB="$LIB"
OUT=gpurun_out/${OUTDIR:-r5}
mkdir -p "$OUT"
B="python3 -u bench.py --steps 20 --warmup 5"
Q="--steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count"
P="timeout -s KILL 120 rocprofv3"
log() { echo "== $(date +%T) $*" >> "$OUT/progress.log"; }
n=0
for s in "$@"; do
  n=$((n + 1))
  log "$s"
  case "$s" in
    tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > "$OUT/gpu_tests.log" 2>&1 ;;
    smoke) timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) timeout -k 10 600 $B > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    bench:*) a="${s#bench:}"; timeout -k 10 600 $B ${a//,/ } > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv \
            -- python3 -u bench.py $Q > "$OUT/prof_c2.log" 2>&1 ;;
    profc4) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv \
              -- python3 -u bench.py --workload C4 $Q > "$OUT/prof_c4.log" 2>&1 ;;
    pmc) $P --pmc FETCH_SIZE -d "$OUT/pmc_calib_fetch" -o p --output-format csv -- ./tools/pmc_calib > "$OUT/pmc1.log" 2>&1 \
         && $P --pmc WRITE_SIZE -d "$OUT/pmc_calib_write" -o p --output-format csv -- ./tools/pmc_calib > "$OUT/pmc2.log" 2>&1 \
         && $P --pmc FETCH_SIZE -d "$OUT/pmc_c2_fetch" -o p --output-format csv -- python3 -u bench.py $Q > "$OUT/pmc3.log" 2>&1 \
         && $P --pmc WRITE_SIZE -d "$OUT/pmc_c2_write" -o p --output-format csv -- python3 -u bench.py $Q > "$OUT/pmc4.log" 2>&1 ;;
    profc2x) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2x" -o run --output-format csv \
              -- python3 -u bench.py --workload C2X $Q > "$OUT/prof_c2x.log" 2>&1 ;;
    pmcc2x) $P --pmc FETCH_SIZE -d "$OUT/pmc_c2x_fetch" -o p --output-format csv -- python3 -u bench.py --workload C2X $Q > "$OUT/pmc9.log" 2>&1 \
            && $P --pmc WRITE_SIZE -d "$OUT/pmc_c2x_write" -o p --output-format csv -- python3 -u bench.py --workload C2X $Q > "$OUT/pmc10.log" 2>&1 ;;
    sqc2x) $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR \
            -d "$OUT/sq_c2x" -o p --output-format csv -- python3 -u bench.py --workload C2X $Q > "$OUT/sq2x.log" 2>&1 ;;
    sqc5) $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR \
            -d "$OUT/sq_c5" -o p --output-format csv -- python3 -u bench.py --workload C5 $Q > "$OUT/sq5.log" 2>&1 ;;
    profc5) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv \
              -- python3 -u bench.py --workload C5 $Q > "$OUT/prof_c5.log" 2>&1 ;;
    pmcc5) $P --pmc FETCH_SIZE -d "$OUT/pmc_c5_fetch" -o p --output-format csv -- python3 -u bench.py --workload C5 $Q > "$OUT/pmc7.log" 2>&1 \
           && $P --pmc WRITE_SIZE -d "$OUT/pmc_c5_write" -o p --output-format csv -- python3 -u bench.py --workload C5 $Q > "$OUT/pmc8.log" 2>&1 ;;
    sqc4) $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_SMEM \
            -d "$OUT/sq_c4" -o p --output-format csv -- python3 -u bench.py --workload C4 $Q > "$OUT/sq1.log" 2>&1 ;;
    sqc4r) $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_SMEM \
             -d "$OUT/sq_c4r" -o p --output-format csv -- python3 -u bench.py --workload C4R $Q > "$OUT/sq2.log" 2>&1 ;;
    pmcc4) $P --pmc FETCH_SIZE -d "$OUT/pmc_c4_fetch" -o p --output-format csv -- python3 -u bench.py --workload C4 $Q > "$OUT/pmc5.log" 2>&1 \
           && $P --pmc WRITE_SIZE -d "$OUT/pmc_c4_write" -o p --output-format csv -- python3 -u bench.py --workload C4 $Q > "$OUT/pmc6.log" 2>&1 ;;
    prof:*) w="${s#prof:}"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${w,,}" -o run --output-format csv \
              -- python3 -u bench.py --workload $w $Q > "$OUT/prof_${w,,}.log" 2>&1 ;;
    pmc:*) w="${s#pmc:}"; $P --pmc FETCH_SIZE -d "$OUT/pmc_${w,,}_fetch" -o p --output-format csv -- python3 -u bench.py --workload $w $Q > "$OUT/pmc_${w,,}_f.log" 2>&1 \
           && $P --pmc WRITE_SIZE -d "$OUT/pmc_${w,,}_write" -o p --output-format csv -- python3 -u bench.py --workload $w $Q > "$OUT/pmc_${w,,}_w.log" 2>&1 ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then log "$s failed rc=$rc"; echo "step $s failed rc=$rc"; exit $rc; fi
done
log done
