# round 5: SIMT efficiency of the step kernels from the hardware (SQ_THREAD_CYCLES_VALU over
# 64 x SQ_ACTIVE_INST_VALU), LDS bank conflicts and store-issue cycles, both shapes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ah; mkdir -p $O
C="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR"
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/s9 -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --check-boards 0 > $O/s9.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/s16 -o p --output-format csv -- python3 bench.py --no-cpu-baseline --shape 16x16x8 --boards 262144 --steps 20 --warmup 5 --check-boards 0 > $O/s16.log 2>&1
echo rc=$?
# and the 16x16 step kernel at 3 waves/SIMD (s163: 168 VGPRs, 599 spilled) vs 2 (the shipped library)
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05ah "libm3_s163.so $S16" "libm3.so $S16" "libm3.so $S16" "libm3_s163.so $S16"
