# round 5, 16x16x8: k_env_step staging rows padded by 16 B (pad: 4-way LDS bank conflicts when a lane
# reads / writes its own 256-B row, instead of 64-way) vs contiguous rows (the shipped library)
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05ai "libm3_pad.so $S16" "libm3.so $S16" "libm3.so $S16" "libm3_pad.so $S16" \
  "libm3_pad.so $S16" "libm3.so $S16"
