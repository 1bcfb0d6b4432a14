# rocprofv3 evidence for bench.py (round 1). Kernel trace/stats and each PMC group in its own pass.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="bench.py --steps 30 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $B > $OUT/kt_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/sq -o sq --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/sq2 -o sq2 --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/sq2.log 2>&1
rc=$?
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
exit $rc
