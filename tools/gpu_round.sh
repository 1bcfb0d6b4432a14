# GPU check: smoke, -m gpu parity suite, bench, and a kernel-trace profile of the bench.
# usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
{ timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; } && \
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --cpu-seconds 8 > $OUT/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > $OUT/kt_bench.log 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
# HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), no trace domains combined
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/write.log 2>&1
