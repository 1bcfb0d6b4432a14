# Phase breakdown (profiling build) + SQ counter passes of the normal build.
# usage: bash tools/gpu_phase.sh <tag>
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 tools/phase_prof.py --shards 1 > $OUT/phase_s1.log 2>&1 && \
timeout -k 10 300 python3 tools/phase_prof.py --shards 4 > $OUT/phase_s4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/sq -o sq --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/sq2 -o sq2 --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/sq2.log 2>&1
