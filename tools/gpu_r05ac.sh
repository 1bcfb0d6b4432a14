# round 5: lean k_env_fix (fx: one board per wave, <= 128 VGPRs, so its waves start beside the
# step waves) vs the 64-lane / 512-VGPR (16x16) one (lz)
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05ac "libm3_fx.so $S16" "libm3_lz.so $S16" "libm3_fx.so" "libm3_lz.so" \
  "libm3_lz.so $S16" "libm3_fx.so $S16" "libm3_lz.so" "libm3_fx.so" "libm3_fx.so $S16" "libm3_lz.so $S16"
