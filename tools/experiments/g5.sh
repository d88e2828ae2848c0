# 4-D full_dp with the K chain summed: GPU tests, then C3 A/B against the
# four-state planes (SK4_NO_GSUM=1), same box.
set -o pipefail
OUT=gpurun_out/g5; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -k "stem4d or 4d or c3 or C3" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', 'parity', l.get('parity',{}).get('max_rel_err'))" $1 "$2"; }
for r in 1 2; do
  SK4_NO_GSUM=1 timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline > $OUT/c3_old_$r.log 2>&1 || { tail -20 $OUT/c3_old_$r.log; exit 1; }
  line $OUT/c3_old_$r.log "c3 4-state r$r"
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline > $OUT/c3_new_$r.log 2>&1 || { tail -20 $OUT/c3_new_$r.log; exit 1; }
  line $OUT/c3_new_$r.log "c3 gsum r$r"
done
timeout -k 10 300 python3 -u bench.py --config c3 > $OUT/c3_cpu.log 2>&1 || { tail -20 $OUT/c3_cpu.log; exit 1; }
line $OUT/c3_cpu.log "c3 gsum with cpu baseline/parity"
