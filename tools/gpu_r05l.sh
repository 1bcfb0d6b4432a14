set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre.so timeout -k 10 300 python3 -u tools/dbg/lanes_env.py 10x8x9 > $O/pre_env_10x8x9.log 2>&1
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre.so timeout -k 10 300 python3 -u tools/dbg/lanes_env.py 12x12x7 > $O/pre_env_12x12x7.log 2>&1
exit 0
