cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r04/fftpmc"; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM -d $OUT/sq -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --sections fft --steps 1 --warmup 0 --no-cpu-baseline --no-verify --no-kernel-profile > $OUT/sq.log 2>&1
echo rc=$?
f=$(find $OUT/sq -name "*counter_collection.csv" | head -1)
python3 "$GRAFT_REPO_ROOT/tools/pmc_kernel_avg.py" "$f" 1 | grep -i persist
rm -f "$f"
