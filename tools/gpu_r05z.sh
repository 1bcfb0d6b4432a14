# round 5, 16x16x8: fifth table round (r5) vs four (ip); ip8 (8 boards per stream wave) again; the
# step kernel with the cascade bounded at 2 + continuation (c16) and at 1 wave/SIMD (w1)
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05z "libm3_r5.so $S16" "libm3_ip.so $S16" "libm3_c16.so $S16" "libm3_w1.so $S16" "libm3_ip8.so $S16" \
  "libm3_ip8.so $S16" "libm3_w1.so $S16" "libm3_c16.so $S16" "libm3_ip.so $S16" "libm3_r5.so $S16"
