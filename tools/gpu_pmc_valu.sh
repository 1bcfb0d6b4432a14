# One PMC pass (VALU/SALU/waves/busy) of bench.py per library variant: bash tools/gpu_pmc_valu.sh <outdir> <lib>...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
for L in "$@"; do
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/$L -o p --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/$L.log 2>&1 || exit 1
done
