set -o pipefail
export TMPDIR=/tmp
for v in "" build/libsk_xnost.so "" build/libsk_xnost.so; do
  SK_LIB_PATH=$v timeout -k 10 400 python3 -u bench.py --config ns --no-cpu-baseline > gpurun_out/v.log 2>&1 || { tail -20 gpurun_out/v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print('ns $v', round(d['value']), round(d['roofline']['kernel_ms_per_launch'],1), round(d['ms_per_step'],1))"
done
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $PWD/gpurun_out/tcc -o run --output-format csv -- python3 $PWD/bench.py --config ns --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/tcc.log 2>&1 || { tail -20 gpurun_out/tcc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/tcc/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if 'dag_stem' in r['Kernel_Name']:
        acc[r['Counter_Name']] += float(r['Counter_Value'])
print(dict(acc))
PY
