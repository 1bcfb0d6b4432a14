# Round evidence for one bench shape, from the driver's own command (python3 bench.py --gpus 1
# --steps 20 --warmup 5; 16x16x8: --shape 16x16x8 --boards 262144): the bench line, a rocprofv3
# kernel trace (--kernel-trace --stats) and one rocprofv3 --pmc pass per counter group, each its
# own run (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE do not fit one pass; <= 8 SQ counters).
# Then: python3 tools/collect_profiles.py gpurun_out/<tag>/<shape> <round-tag>
# usage: bash tools/gpu_profile.sh <tag> [9|16]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-dev}; SH=${2:-9}
if [ "$SH" = 16 ]; then A="--shape 16x16x8 --boards 262144"; O=gpurun_out/$TAG/s16; else A=""; O=gpurun_out/$TAG/s9; fi
mkdir -p $O
B="bench.py --gpus 1 --steps 20 --warmup 5 $A"
timeout -k 10 300 python3 $B > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $B --no-cpu-baseline > $O/kt.log 2>&1 || exit 1
pass() {  # name counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $O/p_$n -o p --output-format csv -- python3 $B --no-cpu-baseline > $O/p_$n.log 2>&1
}
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR || exit 1
pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit 1
echo "profile $TAG s$SH ok"
