#!/bin/bash
# Round-2 (second session) GPU call: parity tests, the full bench line, the
# rocprofv3 kernel trace of the headline, the PMC passes of the headline
# workload.  Every GPU step has its own time limit; the script stops at the
# first failing step.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/r02_bench_prof.sh; rc=$?; echo "benchprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
PMC_NAME=r02b PMC_KEY=coherent_hop_by_hop_1024x256_k8 bash tools/r02_pmc.sh; rc=$?; echo "pmc rc=$rc"
[ $rc -eq 0 ] || exit $rc
# LDS bytes of the Mode P streaming kernel (configs[1] private section), one pass
mkdir -p $OUT/lds
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH \
    SQ_INSTS_LDS_ATOMIC_BANDWIDTH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d /tmp/ldspmc -o p -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --sections private --no-cpu-baseline --no-verify --steps 1 --warmup 0 \
    > "$GRAFT_REPO_ROOT/$OUT/lds/bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/lds/bench.err" )
rc=$?; echo "lds pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_kernel_avg.py /tmp/ldspmc/p_counter_collection.csv 1 > $OUT/lds/avg.jsonl
exit $?
