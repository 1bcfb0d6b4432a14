set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
for i in 1 2; do
for L in pre f2 f2nolr; do
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_$L.so timeout -k 10 300 python3 -u tools/dbg/lanes.py 12x12x7 10x8x9 > $O/${L}_$i.log 2>&1
grep -H failing $O/${L}_$i.log
done; done
exit 0
