# rocprofv3 kernel stats of one coherent run (args: T N K hot [--hbh])
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${TAG:-p} -o run -- python3 tools/coh_bench.py "$@" --no-oracle > gpurun_out/prof/${TAG:-p}.txt 2>&1 || exit 1
