set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre.so timeout -k 10 300 python3 -u tools/dbg/lanes.py > $O/pre.log 2>&1
M3_LIB=$PWD/element-crush-gym_amd/build/libm3.so timeout -k 10 300 python3 -u tools/dbg/lanes.py > $O/cur.log 2>&1
exit 0
