# round-6 GPU session w: chunked shared ring (C5V) — whole suite, default bench line, C5V trace + PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUTDIR=r6w bash tools/gpu_session.sh tests smoke bench prof:C5V pmc:C5V prof:C5
rc=$?
tail -1 gpurun_out/r6w/gpu_tests.log
python3 tools/r6_summ.py gpurun_out/r6w/bench.json
exit $rc
