set -o pipefail
mkdir -p gpurun_out/prof_cfg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in c2 c3 c5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg/$cfg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --no-cpu-baseline > gpurun_out/prof_cfg/$cfg.log 2>&1 || { tail -20 gpurun_out/prof_cfg/$cfg.log; exit 1; }
  tail -1 gpurun_out/prof_cfg/$cfg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["metric"], d["value"], d["roofline"]["kernel_ms_per_launch"], d["roofline"]["launches"])'
done
