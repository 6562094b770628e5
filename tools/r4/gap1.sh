set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/gap1 && mkdir -p $O
Q="--steps 20 --warmup 5 --repeats 1 --no-cpu-baseline --no-fused --extra none --no-list-count"
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/g0 -o run --output-format csv -- ./tools/bin/gap_probe 0 > $O/g0.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/g1 -o run --output-format csv -- ./tools/bin/gap_probe 1 > $O/g1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c4a -o run --output-format csv -- python3 -u bench.py --workload C4 $Q > $O/c4a.log 2>&1 && \
RAFTSTEP_LIB=ablib/lp0/libraftstep.so timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c4b -o run --output-format csv -- python3 -u bench.py --workload C4 $Q > $O/c4b.log 2>&1
