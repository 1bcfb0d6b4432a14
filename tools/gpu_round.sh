# GPU check: smoke, -m gpu parity suite, bench (9x9 headline + 16x16 + rollouts), kernel-trace profile and PMC passes.
# usage: bash tools/gpu_round.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-dev}
shift
XB="$*"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="bench.py --steps 30 --warmup 5 --no-cpu-baseline $XB"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
{ timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ]; } && \
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --cpu-seconds 8 $XB > $OUT/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --cpu-seconds 8 > $OUT/bench16.log 2>&1 && \
timeout -k 10 300 python bench.py --rollouts --steps 5 --warmup 1 > $OUT/rollouts9.log 2>&1 && \
timeout -k 10 300 python bench.py --rollouts --shape 16x16x8 --boards 262144 --steps 3 --warmup 1 > $OUT/rollouts16.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline $XB > $OUT/kt_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt16 -o kt --output-format csv -- python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --no-cpu-baseline > $OUT/kt16_bench.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 $B > $OUT/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 $B > $OUT/write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/sq -o sq --output-format csv -- python3 $B > $OUT/sq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/sq2 -o sq2 --output-format csv -- python3 $B > $OUT/sq2.log 2>&1
