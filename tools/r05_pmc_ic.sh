set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05/ic
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/r05/ic/avail.txt 2>&1 || true
grep -i "icache\|IFETCH\|SQC_" gpurun_out/r05/ic/avail.txt | head -40
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES -d $GRAFT_REPO_ROOT/gpurun_out/r05/ic/p1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/coh_bench.py 1024 256 8 256 --hbh --no-oracle > $GRAFT_REPO_ROOT/gpurun_out/r05/ic/p1.log 2>&1
tail -3 $GRAFT_REPO_ROOT/gpurun_out/r05/ic/p1.log
