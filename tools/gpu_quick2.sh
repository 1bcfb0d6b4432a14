# parity suite + 9x9 and 16x16 bench lines (no profiler). usage: bash tools/gpu_quick2.sh <tag>
set -o pipefail
TAG=${1:-q}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --no-cpu-baseline > $OUT/bench16.log 2>&1
