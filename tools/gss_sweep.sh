set -o pipefail
mkdir -p gpurun_out
for k in ${GSS_KS:-2 4 8}; do
  for c in ${GSS_CFGS:-ns c5}; do
    SK_GSS_K=$k timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline > gpurun_out/gss_${c}_$k.log 2>&1 || { tail -20 gpurun_out/gss_${c}_$k.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/gss_${c}_$k.log').read().strip().splitlines()[-1]); print('$c K=$k', round(d['value']), 'frac', round(d['roofline']['frac'],4), 'ms/launch', round(d['roofline']['kernel_ms_per_launch'],2), 'ms/step', round(d['ms_per_step'],1))"
  done
done
