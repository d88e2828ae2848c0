# NS work-item sizing (SK_GSS_K) around 1.0, alternating, two rounds.
set -o pipefail
OUT=gpurun_out/g21; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
for r in 1 2; do
  for k in 0.75 1.0 1.5; do
    SK_GSS_K=$k timeout -k 10 300 python3 -u bench.py --config ns --no-cpu-baseline > $OUT/ns_${k}_$r.log 2>&1 || { tail -20 $OUT/ns_${k}_$r.log; exit 1; }
    line $OUT/ns_${k}_$r.log "ns gss_k=$k r$r"
  done
done
for k in 1.0; do
  SK_GSS_K=$k timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline > $OUT/c5_$k.log 2>&1 || { tail -20 $OUT/c5_$k.log; exit 1; }
  line $OUT/c5_$k.log "c5 gss_k=$k"
done
