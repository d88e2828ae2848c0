set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_bench.sh ns r02f_ns --no-tests || exit 1
bash tools/gpu_bench.sh c3 r02f_c3 --no-tests || exit 1
