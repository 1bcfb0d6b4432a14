# round 5, 9x9x6: two-stage prefetch reset with rejection sampling (t9: 4 resets per stream wave,
# accepted tiles compacted by ballot + mbcnt, 7-8 rounds per table row) vs k_init + k_init_coop (lz)
FAST=1 bash tools/gpu_ab.sh r05af "libm3_t9.so" "libm3_lz.so" "libm3_lz.so" "libm3_t9.so" "libm3_t9.so" "libm3_lz.so"
