# round 5: legal sets derived on request (lz, lz8) vs written every step (r5); 4 vs 8 boards per
# stream wave with five table rounds
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05aa "libm3_lz.so" "libm3_r5.so" "libm3_lz.so $S16" "libm3_lz8.so $S16" "libm3_r5.so $S16" \
  "libm3_r5.so" "libm3_lz.so" "libm3_r5.so $S16" "libm3_lz8.so $S16" "libm3_lz.so $S16" \
  "libm3_lz.so" "libm3_r5.so" "libm3_lz.so $S16" "libm3_lz8.so $S16" "libm3_r5.so $S16"
