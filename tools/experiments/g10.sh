# New 4-D test; NS host planning times per step (SK_HOST_STATS).
set -o pipefail
OUT=gpurun_out/g10; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stem4d.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
SK_HOST_STATS=1 timeout -k 10 300 python3 -u bench.py --config ns --steps 3 --warmup 1 --no-cpu-baseline > $OUT/ns.log 2>&1 || { tail -20 $OUT/ns.log; exit 1; }
grep -E "^\[host\]" $OUT/ns.log | tail -8
tail -1 $OUT/ns.log | cut -c1-200
