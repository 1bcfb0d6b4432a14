set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre.so timeout -k 10 300 python3 -u tools/dbg/lanes_k.py 10x8x9 > $O/pre_k.log 2>&1
exit 0
