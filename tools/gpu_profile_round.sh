#!/bin/bash
# Round profile of the default bench workload: rocprofv3 kernel-trace stats,
# then the PMC passes (separate runs), then a JSON summary.
#   PROF_NAME (default r01), PROF_ARGS (default "--steps 3 --warmup 1 --no-cpu-baseline")
cd "$GRAFT_REPO_ROOT" || exit 1
NAME=${PROF_NAME:-r01}
PROF_NAME=$NAME PROF_ARGS=${PROF_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --coherent-tiles 0"} bash tools/gpu_prof.sh || exit $?
PMC_NAME=$NAME PMC_ARGS=${PMC_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline --no-verify --coherent-tiles 0"} bash tools/gpu_pmc.sh || exit $?
cd "$GRAFT_REPO_ROOT"
python3 tools/pmc_summary.py gpurun_out/prof/$NAME/run_kernel_stats.csv gpurun_out/pmc/$NAME gpurun_out/prof/${NAME}_summary.json "$NAME" ${PROF_TILES:-1024} ${PROF_PER_TILE:-1048576}
