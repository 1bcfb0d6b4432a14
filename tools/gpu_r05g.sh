set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
grep -i -E "ICACHE|IFETCH|SQC_|INST_LEVEL|WAIT_INST|SQ_INSTS_BRANCH|SQ_INSTS_SMEM|LEVEL" $O/counters.txt | head -100 > $O/counters_sel.txt
exit 0
