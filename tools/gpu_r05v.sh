# round 5: counter zeroing by the blocks with work only (zc) vs every block (gd) at 9x9; two-stage
# 16x16x8 reset with U=4 interleave at G = 8 (zc) / 16 (g16) / 4 (g4) boards per wave vs
# k_init_fix_lane (fl); kernel traces of zc at both shapes
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05v "libm3_zc.so" "libm3_gd.so" "libm3_zc.so $S16" "libm3_g16.so $S16" "libm3_g4.so $S16" \
  "libm3_fl.so $S16" "libm3_gd.so" "libm3_zc.so" "libm3_fl.so $S16" "libm3_g4.so $S16" "libm3_g16.so $S16" "libm3_zc.so $S16" &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_zc.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05v/kt16 -o kt -- \
  python3 bench.py $S16 --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > gpurun_out/r05v/kt16.log 2>&1 &&
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_zc.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05v/kt9 -o kt -- \
  python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > gpurun_out/r05v/kt9.log 2>&1
