# round 5: stream stage with the second block twisted in place (ip: 4 boards per wave, ip8: 8; 10 / 20 KB
# of LDS) vs out of place (zk: 4 boards, 16 KB)
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05y "libm3_ip.so $S16" "libm3_ip8.so $S16" "libm3_zk.so $S16" \
  "libm3_zk.so $S16" "libm3_ip8.so $S16" "libm3_ip.so $S16" "libm3_ip.so" "libm3_zk.so"
