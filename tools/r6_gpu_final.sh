# round-6 final evidence session: whole GPU suite, smoke, the default bench line, kernel traces and PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUTDIR=r6final3 bash tools/gpu_session.sh tests smoke bench prof profc4 prof:C2S prof:C4S prof:C5V profc2x pmc pmcc4 pmcc2x pmcc5 pmc:C2S pmc:C4S pmc:C5V
rc=$?
tail -1 gpurun_out/r6final3/gpu_tests.log
python3 tools/r6_summ.py gpurun_out/r6final3/bench.json
exit $rc
