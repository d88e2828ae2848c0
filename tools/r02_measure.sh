#!/bin/bash
# r02 measurement round trip (run through gpurun from the repo root):
# GPU parity suite, smoke, NS bench line + rocprofv3 kernel stats, C4 bench
# line + kernel stats + VALU/LDS counters of the BPLA kernel.
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd); OUT=gpurun_out/r02
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for c in ns c4; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_$c -o run -- python3 $ROOT/bench.py --config $c --no-cpu-baseline > $OUT/prof_$c.log 2>&1 || { tail -20 $OUT/prof_$c.log; exit 1; }
  db=$(find $OUT/prof_$c -name "*.db" -print -quit)
  python3 tools/rocpd_stats.py $db $OUT/${c}_kernel_stats.csv && head -4 $OUT/${c}_kernel_stats.csv | cut -c1-120
  tail -1 $OUT/prof_$c.log > $OUT/prof_${c}_line.json
  timeout -k 10 500 python3 -u bench.py --config $c > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | cut -c1-200
done
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $ROOT/$OUT/pmc_c4 -o run --output-format csv -- python3 $ROOT/bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_c4.log 2>&1 || { tail -20 $OUT/pmc_c4.log; exit 1; }
python3 tools/pmc_sum.py $OUT/pmc_c4 sk_bpla > $OUT/pmc_c4.json && cat $OUT/pmc_c4.json
tail -1 $OUT/pmc_c4.log | cut -c1-200
