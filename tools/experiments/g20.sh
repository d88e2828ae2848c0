# NS: work-item sizing (SK_GSS_K) sweep on the final tree; C4 chunk sweep (SK_BPLA_CHUNK).
set -o pipefail
OUT=gpurun_out/g20; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
for k in 1.5 1.0 2.0 3.0 1.5; do
  SK_GSS_K=$k timeout -k 10 300 python3 -u bench.py --config ns --no-cpu-baseline > $OUT/ns_$k.log 2>&1 || { tail -20 $OUT/ns_$k.log; exit 1; }
  line $OUT/ns_$k.log "ns gss_k=$k"
done
for c in 0 4 8 12; do
  SK_BPLA_CHUNK=$c timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu-baseline > $OUT/c4_$c.log 2>&1 || { tail -20 $OUT/c4_$c.log; exit 1; }
  line $OUT/c4_$c.log "c4 chunk=$c"
done
