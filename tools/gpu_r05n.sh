set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_f2nolr.so timeout -k 10 300 python3 -u tools/dbg/lanes.py > $O/f2nolr.log 2>&1
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_f2.so timeout -k 10 300 python3 -u tools/dbg/lanes.py 12x12x7 > $O/f2_again.log 2>&1
exit 0
