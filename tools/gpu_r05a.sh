# round 5, first look: phase profile of the step kernels (fast prof build) + a baseline bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/phase_prof.py --shards 2 --steps 20 > $OUT/phase9.log 2>&1 &&
timeout -k 10 300 python3 -u tools/phase_prof.py --shards 2 --steps 20 --boards 262144 --shape 16x16x8 > $OUT/phase16.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 64 > $OUT/bench9.log 2>&1
