# round 5, 9x9x6: k_init's lockstep draw budget before a prefetch reset is deferred to k_init_coop
# (M3_RESET_KCAP 400 / 454 (lz, shipped) / 520)
FAST=1 bash tools/gpu_ab.sh r05ab "libm3_kc400.so" "libm3_lz.so" "libm3_kc520.so" \
  "libm3_kc520.so" "libm3_lz.so" "libm3_kc400.so" "libm3_lz.so" "libm3_kc400.so" "libm3_kc520.so"
