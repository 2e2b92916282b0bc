cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/probe
timeout -k 10 600 python -u -m pytest tests/test_gpu_coherent.py tests/test_gpu_noc.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/probe/tests.txt 2>&1 || { tail -30 gpurun_out/probe/tests.txt; exit 1; }
tail -2 gpurun_out/probe/tests.txt
timeout -k 10 300 python -u tools/coh_bench.py 1024 256 8 256 --hbh --no-oracle 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/coh_bench.py 1024 1024 8 256 --no-oracle 2>&1 | grep -v amdgpu.ids
export TMPDIR=/tmp
TAG=hbh bash tools/r02_prof.sh 1024 256 8 256 --hbh
