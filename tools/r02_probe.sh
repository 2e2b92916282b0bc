cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/probe
export GG_COH_PROFILE=1
timeout -k 10 240 python -u tools/coh_bench.py 1024 1024 8 256 --no-oracle > gpurun_out/probe/hc1024.txt 2>&1 || exit 1
timeout -k 10 240 python -u tools/coh_bench.py 256 512 1 64 --no-oracle > gpurun_out/probe/hc256.txt 2>&1 || exit 1
