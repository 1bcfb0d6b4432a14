# round 5: per-board chain word of the current episode (mc: the step's RNG words load with the board,
# before the staging barrier) vs the per-slot word behind the slot byte (lz)
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05ag "libm3_mc.so" "libm3_lz.so" "libm3_mc.so $S16" "libm3_lz.so $S16" \
  "libm3_lz.so" "libm3_mc.so" "libm3_lz.so $S16" "libm3_mc.so $S16" "libm3_mc.so" "libm3_lz.so"
