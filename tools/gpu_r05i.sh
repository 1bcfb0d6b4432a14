set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
export M3_LIB=$PWD/element-crush-gym_amd/build/libm3_base.so
for cfg in "--shards 2" "--shards 3" "--shards 4 --hw-queues 16" "--shards 3 --hw-queues 16" "--shards 6 --hw-queues 16" "--shards 8 --hw-queues 24"; do
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 $cfg > $O/b.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print('$cfg', '%.4g'%d['value'], '%.3f'%d['ms_per_step'])"
done
