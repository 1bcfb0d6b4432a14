# Throughput vs shard count (HIP streams per GPU) and the step-only cost (no autoreset, diagnostic).
# usage: bash tools/shard_sweep.sh <tag>
set -o pipefail
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
summ() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], '%.4g env-steps/s  %.3f ms/step  kernel %.3f ms x %d boards' % (d['value'], d['ms_per_step'], r['avg_kernel_ms'], r['boards_per_launch']))" $1 "$2"; }
for s in 1 2 4 8; do
  timeout -k 10 200 python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline --shards $s > $OUT/s$s.log 2>&1 || exit 1
  summ $OUT/s$s.log "shards=$s"
done
for s in 1 4; do
  timeout -k 10 200 python3 bench.py --steps 19 --warmup 1 --no-cpu-baseline --shards $s --no-autoreset > $OUT/nr$s.log 2>&1 || exit 1
  summ $OUT/nr$s.log "no-autoreset shards=$s"
done
