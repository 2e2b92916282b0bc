#!/bin/bash
# Round-6 quick traffic check of library variants: one rocprofv3 FETCH_SIZE
# pass and one SQ instruction pass of the bench headline (one run) per
# variant (VARIANTS: "base" = the tree's build, else a .so path); prints each
# kernel's mean FETCH_SIZE (KiB, uncalibrated) and VALU / SALU per launch.
# PASSES="name:CTR CTR|name2:..." replaces the two passes; BENCH_ARGS extends the bench command.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r06/${TAG:-fetch}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=""; name=base; else lib=$GRAFT_REPO_ROOT/$v; name=$(basename $(dirname $v)); fi
  IFS='|' read -ra PL <<< "${PASSES:-fetch:FETCH_SIZE|sq:SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY}"
  for pass in "${PL[@]}"; do
    GG_LIB=$lib timeout -k 10 300 rocprofv3 --pmc ${pass#*:} -d "$OUT/$name/${pass%%:*}" -o run --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --sections "" --steps 1 --warmup 0 --no-cpu-baseline --no-verify \
      --no-kernel-profile $BENCH_ARGS > "$OUT/$name.${pass%%:*}.log" 2>&1 || { echo "pass $name ${pass%%:*} failed"; tail -5 "$OUT/$name.${pass%%:*}.log"; exit 1; }
  done
  python3 - "$OUT/$name" "$name" <<'PY'
import collections, csv, glob, os, sys
d, name = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, 0]))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        a = acc[k][r["Counter_Name"]]; a[0] += float(r["Counter_Value"]); a[1] += 1
for k, c in sorted(acc.items()):
    n = max(x[1] for x in c.values())
    if n < int(os.environ.get("MINL", "100")): continue
    print(name, k, "launches~%d" % n, " ".join("%s=%.1f" % (m, s / max(cnt, 1)) for m, (s, cnt) in sorted(c.items())))
PY
  find "$OUT/$name" -name "*counter_collection.csv" -delete
done
exit 0
