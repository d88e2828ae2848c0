#!/bin/bash
# BPLA iteration on the GPU box: BPLA parity tests, the C4 bench line and the
# kernel's instruction counters.  Usage: tools/c4_iter.sh TAG [extra pytest files...]
set -o pipefail
TAG=${1:-c4}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bpla.py tests/test_bpla_grad.py tests/test_bpla_schedule.py tests/test_large_configs.py "$@" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 -u bench.py --config c4 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 -c "import json,sys; l=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); r=l['roofline']; print('C4', round(l['value']), 'pairs/s', round(r['kernel_ms_per_launch'],3), 'ms/launch frac', round(r['frac'],4), 'parity', l['parity']['max_rel_err'])"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $PWD/$OUT/pmc -o run --output-format csv -- python3 $PWD/bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
python3 tools/pmc_sum.py $OUT/pmc sk_bpla_fast > $OUT/pmc.json && cat $OUT/pmc.json
python3 -c "import json; c=json.load(open('$OUT/pmc.json')); l=json.loads([x for x in open('$OUT/pmc.log') if x.startswith('{')][-1]); n=l['cells_per_step']; print('per cell: VALU %.2f SALU %.2f LDS %.2f' % (c['SQ_INSTS_VALU']*64/n, c['SQ_INSTS_SALU']*64/n, c['SQ_INSTS_LDS']*64/n))"
