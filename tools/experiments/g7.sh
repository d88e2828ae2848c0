# C5 and C2 measured on the current tree; the C3 bench line with its regenerated traffic profile.
set -o pipefail
bash tools/measure.sh c5 r03q_c5 && bash tools/measure.sh c2 r03q_c2 || exit 1
mkdir -p gpurun_out/r03q_c3b
timeout -k 10 500 python3 -u bench.py --config c3 > gpurun_out/r03q_c3b/bench.log 2>&1 || { tail -20 gpurun_out/r03q_c3b/bench.log; exit 1; }
tail -1 gpurun_out/r03q_c3b/bench.log | cut -c1-300
