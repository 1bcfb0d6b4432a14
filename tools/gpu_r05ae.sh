# round 5, 9x9x6: k_env_step at 3 waves/SIMD (sw3: 135 VGPRs, no spill) vs 4 (lz: 128, 6 spilled, reloaded
# from scratch behind s_waitcnt vmcnt(0) at loop exits)
FAST=1 bash tools/gpu_ab.sh r05ae "libm3_sw3.so" "libm3_lz.so" "libm3_lz.so" "libm3_sw3.so" "libm3_sw3.so" "libm3_lz.so"
