# 4-D K-sum kernel: rows fetched one vs two ahead (C3 A/B), after the 4-D GPU tests.
set -o pipefail
OUT=gpurun_out/g9; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
SK_LIB_PATH=$PWD/build/libsk_pf2.so timeout -k 10 500 python -u -m pytest tests -m gpu -k "stem4d" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline > $OUT/c3_pf1_$r.log 2>&1 || { tail -20 $OUT/c3_pf1_$r.log; exit 1; }
  line $OUT/c3_pf1_$r.log "c3 pf1 r$r"
  SK_LIB_PATH=$PWD/build/libsk_pf2.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline > $OUT/c3_pf2_$r.log 2>&1 || { tail -20 $OUT/c3_pf2_$r.log; exit 1; }
  line $OUT/c3_pf2_$r.log "c3 pf2 r$r"
done
