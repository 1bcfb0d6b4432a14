set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
export M3_LIB=$PWD/element-crush-gym_amd/build/libm3_base.so
B="bench.py --steps 8 --warmup 2 --no-cpu-baseline --check-boards 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_WAIT_INST_LDS -d $O/p1 -o p1 --output-format csv -- python3 $B > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d $O/p2 -o p2 --output-format csv -- python3 $B > $O/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM -d $O/p3 -o p3 --output-format csv -- python3 $B > $O/p3.log 2>&1
