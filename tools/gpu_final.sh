# Round evidence for both bench shapes: smoke, the -m gpu suite, bench lines (9x9x6 headline
# with the CPU baseline, 16x16x8, rollouts), a rocprofv3 kernel trace of each bench command
# and the PMC passes (one rocprofv3 run per counter group) that profiles/traffic*.json derive from.
# usage: [SKIP_TESTS=1] bash tools/gpu_final.sh <tag>     (then: tools/collect_profiles.py gpurun_out/<tag>/s9 <tag>,
#                                                  tools/collect_profiles.py gpurun_out/<tag>/s16 <tag>_16x16x8)
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O/s9 $O/s16
S16="--shape 16x16x8 --boards 262144"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
{ [ -n "$SKIP_TESTS" ] || { timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ]; }; } && \
timeout -k 10 300 python3 bench.py > $O/s9/bench.log 2>&1 && \
timeout -k 10 300 python3 bench.py $S16 --steps 40 --warmup 10 > $O/s16/bench.log 2>&1 && \
timeout -k 10 300 python3 bench.py --rollouts --steps 5 --warmup 1 > $O/rollouts9.log 2>&1 && \
timeout -k 10 300 python3 bench.py --rollouts $S16 --steps 3 --warmup 1 > $O/rollouts16.log 2>&1 && \
for s in s9 s16; do
  if [ $s = s9 ]; then A="--steps 60 --warmup 10"; else A="$S16 --steps 40 --warmup 10"; fi
  B="bench.py --no-cpu-baseline $A"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$s/kt -o kt --output-format csv -- python3 $B > $O/$s/kt.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/$s/fetch -o fetch --output-format csv -- python3 $B > $O/$s/fetch.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/$s/write -o write --output-format csv -- python3 $B > $O/$s/write.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/$s/sq -o sq --output-format csv -- python3 $B > $O/$s/sq.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/$s/sq2 -o sq2 --output-format csv -- python3 $B > $O/$s/sq2.log 2>&1 || exit 1
done
