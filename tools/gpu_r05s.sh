# round 5: parity-gated A/B of the decomposed gravity (gd, default) vs the per-row loop (gl)
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05s "libm3_gd.so" "libm3_gl.so" "libm3_gd.so $S16" "libm3_gl.so $S16" \
  "libm3_gl.so" "libm3_gd.so" "libm3_gl.so $S16" "libm3_gd.so $S16"
