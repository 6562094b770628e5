set -o pipefail
cd /root/repo; export TMPDIR=/tmp; O=gpurun_out/c5chk; mkdir -p $O
timeout -k 10 120 python -u bench.py --workload C5 --steps 100 --warmup 5 --no-cpu-baseline > $O/b1.log 2>&1 \
&& timeout -k 10 180 rocprofv3 --kernel-trace --stats -T -d $O/prof -o run --output-format csv -- python3 -u bench.py --workload C5 --steps 100 --warmup 5 --no-cpu-baseline > $O/p.log 2>&1 \
&& timeout -k 10 120 python -u bench.py --workload C5 --steps 100 --warmup 5 --no-cpu-baseline > $O/b2.log 2>&1 \
&& timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/b3.log 2>&1
