# kernel trace of a short 9x9 bench + phase profile (profiling build). usage: bash tools/gpu_trace.sh <tag>
set -o pipefail
TAG=${1:-tr}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline > $OUT/kt_bench.log 2>&1 && \
timeout -k 10 300 python3 tools/phase_prof.py --shards 1 > $OUT/phase.log 2>&1
