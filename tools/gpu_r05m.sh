set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre_wps1.so timeout -k 10 300 python3 -u tools/dbg/lanes.py > $O/pre_wps1.log 2>&1
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_f2.so timeout -k 10 300 python3 -u tools/dbg/lanes.py > $O/cur_wps2.log 2>&1
exit 0
