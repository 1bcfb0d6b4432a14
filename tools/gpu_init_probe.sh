set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/initprobe
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o kt --output-format csv -- python3 tools/init_probe.py > $OUT/probe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc -o pmc --output-format csv -- python3 tools/init_probe.py > $OUT/pmc.log 2>&1
