# PMC passes (one rocprofv3 run per counter group) of bench.py for one library variant.
# usage: bash tools/gpu_pmc.sh <outdir> <lib> [bench args]
set -o pipefail
export TMPDIR=/tmp
O=$1; L=$2; shift 2
mkdir -p $O
export M3_LIB=$PWD/element-crush-gym_amd/build/$L
B="bench.py --steps 8 --warmup 2 --no-cpu-baseline $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o p1 --output-format csv -- python3 $B > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT -d $O/p2 -o p2 --output-format csv -- python3 $B > $O/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o p3 --output-format csv -- python3 $B > $O/p3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o p4 --output-format csv -- python3 $B > $O/p4.log 2>&1
