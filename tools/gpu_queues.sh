# Throughput vs board shards (HIP streams) and hardware queues. usage: bash tools/gpu_queues.sh <tag> "q:s q:s ..."
set -o pipefail
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for qs in $2; do
  q=${qs%%:*}; s=${qs##*:}
  timeout -k 10 200 python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline --shards $s --hw-queues $q > $OUT/q${q}s${s}.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('$OUT/q${q}s${s}.log').read().strip().splitlines()[-1]);print('q=$q shards=$s %.4g env-steps/s %.3f ms/step kernel %.3f ms' % (d['value'], d['ms_per_step'], d['roofline']['avg_kernel_ms']))"
done
