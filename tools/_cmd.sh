set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_bench.sh c5 r02f_c5 --no-tests || exit 1
bash tools/gpu_bench.sh c2 r02f_c2 --no-tests || exit 1
bash tools/gpu_bench.sh c4 r02f_c4 --no-tests || exit 1
