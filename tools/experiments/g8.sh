# BPLA: row-B sums carried across steps (A/B against the HEAD library), after the BPLA GPU tests.
set -o pipefail
OUT=gpurun_out/g8; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -k "bpla or BPLA" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u tools/bpla_prec.py > $OUT/prec.log 2>&1 || { tail -20 $OUT/prec.log; exit 1; }
cat $OUT/prec.log | grep default
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value']), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
for r in 1 2 3; do
  SK_LIB_PATH=$PWD/build/libsk_c4base.so timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu-baseline > $OUT/c4_old_$r.log 2>&1 || { tail -20 $OUT/c4_old_$r.log; exit 1; }
  line $OUT/c4_old_$r.log "c4 base r$r"
  timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu-baseline > $OUT/c4_new_$r.log 2>&1 || { tail -20 $OUT/c4_new_$r.log; exit 1; }
  line $OUT/c4_new_$r.log "c4 sums carried r$r"
done
