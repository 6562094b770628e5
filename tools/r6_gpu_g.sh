# round-6 GPU session g: PMC passes (tools/pmc_all.sh) + list-kernel wave phases (diagnostics build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUTDIR=r6g bash tools/gpu_session.sh bench pmc pmcc4 pmcc2x pmcc5 pmc:C2S pmc:C4S || exit 1
RAFTSTEP_LIB=tools/bin/wprof/libraftstep.so timeout -k 10 200 python -u tools/list_prof.py > gpurun_out/r6g/list_prof_c4.log 2>&1; tail -20 gpurun_out/r6g/list_prof_c4.log
RAFTSTEP_LIB=tools/bin/wprof/libraftstep.so timeout -k 10 200 python -u tools/list_prof.py --workload C4S > gpurun_out/r6g/list_prof_c4s.log 2>&1; tail -20 gpurun_out/r6g/list_prof_c4s.log
