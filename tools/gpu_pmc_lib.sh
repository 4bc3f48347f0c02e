#!/bin/bash
# One SQ counter pass of the draw alone (bench --no-pairs) per library build: LABEL:LIB entries.
# Usage (repo root, GPU box): bash tools/gpu_pmc_lib.sh "k0:exp/k0/lib.so tree:" [bench args...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/pmc_lib; mkdir -p "$OUT"
ENTRIES=$1; shift || true
export TMPDIR=/tmp
cd /tmp
for ent in $ENTRIES; do
  label=${ent%%:*}; lib=${ent#*:}
  if [ -n "$lib" ]; then export CSA_LIB=$ROOT/$lib; else unset CSA_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
      -d "$OUT/$label" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --iso-steps 0 --no-pairs \
      --no-cpu-baseline --no-api "$@" > "$OUT/$label.json" 2> "$OUT/$label.err" || { echo "rc=$? $label"; tail -3 "$OUT/$label.err"; exit 1; }
  python3 - "$OUT/$label" "$label" <<'PY'
import csv, glob, sys, collections
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/run_counter_collection.csv', recursive=True)[0])))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    if 'draw_' not in r['Kernel_Name']: continue
    acc[r['Kernel_Name'][:60]][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in acc.items():
    print(sys.argv[2], k, {c: '%.4g' % x for c, x in sorted(v.items())})
PY
done
