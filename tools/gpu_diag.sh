#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 100 python3 -u tools/ab.py --ticks 200 --rounds 5 base: > $OUT/diag1.log 2>&1 \
&& timeout -k 10 100 python3 -u tools/ab.py --noprof --ticks 200 --rounds 5 base: > $OUT/diag2.log 2>&1 \
&& timeout -k 10 100 python3 -u tools/ab.py --ticks 400 --rounds 5 --groups 65536 base: se1:RAFTSTEP_SLOW_EVERY=1 > $OUT/diag3.log 2>&1 \
&& timeout -k 10 100 python3 -u tools/ab.py --noprof --ticks 400 --rounds 5 --groups 65536 base: > $OUT/diag4.log 2>&1 \
&& timeout -k 10 120 ./raft-sample_amd/lib/raft_cluster --mode tick --entries 2000 > $OUT/cluster_tick.log 2>&1 \
&& timeout -k 10 200 ./raft-sample_amd/lib/raft_cluster --mode handlers --entries 2000 > $OUT/cluster_handlers.log 2>&1
