set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre_ucas.so timeout -k 10 300 python3 -u tools/dbg/lanes.py 12x12x7 10x8x5 10x8x9 > $O/pre_ucas.log 2>&1
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre_ucas.so timeout -k 10 300 python3 -u tools/dbg/lanes_k.py 10x8x9 > $O/pre_ucas_k.log 2>&1
exit 0
