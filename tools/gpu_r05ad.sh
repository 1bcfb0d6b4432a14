# round 5, 9x9x6: k_env_cont_grid at 3 waves/SIMD (cw3: 168 VGPRs, 43 spilled) vs 4 (lz: 128, 98 spilled)
FAST=1 bash tools/gpu_ab.sh r05ad "libm3_cw3.so" "libm3_lz.so" "libm3_lz.so" "libm3_cw3.so" "libm3_cw3.so" "libm3_lz.so"
