#!/bin/bash
# One measurement round trip on the GPU box (run from the repo root through
# gpurun):  [GPU parity suite + smoke], rocprofv3 kernel trace + stats of the
# bench, FETCH_SIZE / WRITE_SIZE / LDS counter passes (one rocprofv3 run
# each), tools/profile_summary.py -> profiles/<config>_traffic.json (stamped
# with the source hash), then the plain bench line, which reads that file.
# Usage: tools/measure.sh CONFIG TAG [--tests]
set -o pipefail
CFG=${1:-ns}; TAG=${2:-$CFG}; TESTS=$3
ROOT=$(pwd); OUT=gpurun_out/$TAG
case $CFG in
  ns) KIND=ss; KSUB=sk_dag_stem_kernel;;
  c2) KIND=ss; KSUB=sk_dag_stem_kernel;;
  c5) KIND=stem; KSUB=sk_dag_stem_kernel;;
  c3) KIND=stem4d; KSUB=sk_stem4d;;
  c4) KIND=bpla; KSUB=sk_bpla_fast;;
  *) echo "unknown config $CFG"; exit 2;;
esac
mkdir -p $OUT; export TMPDIR=/tmp
if [ "$TESTS" == "--tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --config $CFG --no-cpu-baseline > $OUT/bench_prof.log 2>&1 || { tail -20 $OUT/bench_prof.log; exit 1; }
echo trace_done
run_pmc() {  # name counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $ROOT/$OUT/$name -o run --output-format csv -- \
    python3 $ROOT/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  echo ${name}_done
}
run_pmc FETCH_SIZE FETCH_SIZE || exit 1
run_pmc WRITE_SIZE WRITE_SIZE || exit 1
run_pmc LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE || exit 1
python3 tools/profile_summary.py $OUT $CFG $KSUB $OUT/${CFG}_traffic.json > $OUT/summary.log 2>&1 || { tail -20 $OUT/summary.log; exit 1; }
cp $OUT/${CFG}_traffic.json profiles/${CFG}_traffic.json
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
timeout -k 10 500 python3 -u bench.py --config $CFG > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
