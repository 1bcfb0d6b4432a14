# round 5, shipped library: the 9x9 rollout line (its k_rollout shares the 6-slot group table)
set -o pipefail
mkdir -p gpurun_out/r05ro
timeout -k 10 300 python3 bench.py --rollouts --steps 5 --warmup 1 > gpurun_out/r05ro/rollouts9.log 2>&1
echo rc=$?; grep "^{" gpurun_out/r05ro/rollouts9.log | tail -c 400
