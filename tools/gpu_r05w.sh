# round 5: counter blocks zeroed by the previous step's k_env_fix (zk, CBLOCKS = 4) vs the
# tickets of the blocks with work (zc); 16x16 with G = 4 in both zk and g4
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05w "libm3_zk.so" "libm3_zc.so" "libm3_zk.so $S16" "libm3_g4.so $S16" \
  "libm3_zc.so" "libm3_zk.so" "libm3_g4.so $S16" "libm3_zk.so $S16"
