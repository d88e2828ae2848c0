# HBM bytes per cell and time of DAG-kernel library variants on one config:
# tools/_nt.sh TAG CONFIG lib...   ("-" = in-tree build)
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1)); L=""; [ "$lib" != "-" ] && L="$PWD/$lib"
  for c in FETCH_SIZE WRITE_SIZE; do
    SK_LIB_PATH=$L timeout -s KILL 300 rocprofv3 --pmc $c -d $PWD/$OUT/${i}_$c -o run --output-format csv -- \
      python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > $OUT/${i}_$c.log 2>&1 || { tail -20 $OUT/${i}_$c.log; exit 1; }
  done
  python3 - $OUT $i "$lib" <<'PY'
import json, subprocess, sys
out, i, lib = sys.argv[1:4]
f = json.loads(subprocess.check_output(["python3", "tools/pmc_sum.py", f"{out}/{i}_FETCH_SIZE", "sk_dag_stem_kernel"]))
w = json.loads(subprocess.check_output(["python3", "tools/pmc_sum.py", f"{out}/{i}_WRITE_SIZE", "sk_dag_stem_kernel"]))
line = [l for l in open(f"{out}/{i}_FETCH_SIZE.log") if l.startswith('{"metric"')][-1]
cells = json.loads(line)["cells_per_step"]
rd, wr = 2048.0 * f["FETCH_SIZE"] / cells, 1024.0 * w["WRITE_SIZE"] / cells
print(f"{lib}: read {rd:.2f} write {wr:.2f} total {rd + wr:.2f} B/cell")
PY
done
