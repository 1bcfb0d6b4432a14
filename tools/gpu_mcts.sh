# GPU check of the rollout path: -m gpu MCTS tests + the rollout bench (both shapes).
# usage: bash tools/gpu_mcts.sh <tag>
set -o pipefail
TAG=${1:-mcts}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_mcts.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --rollouts --steps 5 --warmup 1 > $OUT/bench9.log 2>&1 && \
timeout -k 10 300 python bench.py --rollouts --shape 16x16x8 --boards 262144 --steps 3 --warmup 1 > $OUT/bench16.log 2>&1
