# round 5, 9x9x6: 6 match-group slots in LDS per lane (g6: 9 KB per wave) vs 4 (the shipped library,
# 6 KB; more groups spill to the global pool)
FAST=1 bash tools/gpu_ab.sh r05aj "libm3_g6.so" "libm3.so" "libm3.so" "libm3_g6.so" "libm3_g6.so" "libm3.so"
