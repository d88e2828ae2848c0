# 4-D pre-combined kernel: rows two ahead (in-tree) vs one ahead (4 waves per SIMD) vs two ahead capped at 128 VGPRs.
set -o pipefail
OUT=gpurun_out/g16; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
for r in 1 2; do
  for v in - prepf1 premb4; do
    L=""; [ "$v" != "-" ] && L="$PWD/build/libsk_$v.so"
    SK_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline > $OUT/c3_${v}_$r.log 2>&1 || { tail -20 $OUT/c3_${v}_$r.log; exit 1; }
    line $OUT/c3_${v}_$r.log "c3 $v r$r"
  done
done
