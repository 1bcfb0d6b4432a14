set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05e
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/phase_prof.py --shards 2 --steps 20 > $OUT/phase9.log 2>&1
