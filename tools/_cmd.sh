set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_stem4d.py -m gpu > gpurun_out/pytest_s4d.log 2>&1 || { tail -30 gpurun_out/pytest_s4d.log; exit 1; }
tail -3 gpurun_out/pytest_s4d.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ali -o ali -- python3 -u tools/probe_perf.py 200 24 stem4d_ali > gpurun_out/probe_ali.log 2>&1 || { tail -20 gpurun_out/probe_ali.log; exit 1; }
grep "pairs/s" gpurun_out/probe_ali.log
find gpurun_out/prof_ali -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -8
