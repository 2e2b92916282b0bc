# GPU parity tests of the round-2 engine (one pytest process, per-test timeout)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/r02/pytest_gpu.log; exit $rc
