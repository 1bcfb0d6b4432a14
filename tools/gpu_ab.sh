# Parity-gated A/B bench of library variants x bench options (9x9x6 headline config unless
# the spec passes --shape). A variant is timed only after the bit-exactness suite passes
# against it (tests/test_gpu_parity.py + test_gpu_env.py with M3_LIB pointing at the variant);
# a variant that fails is reported as REJECTED and never timed.
# PARITY_TESTS overrides the gating test files (e.g. for a library built before a test existed).
# FAST=1: the libraries are headline-only builds (make variant-fast: 9x9x6 and 16x16x8 only), so the
# gate is test_gpu_parity.py + test_gpu_checkpoint.py + the headline-shape cases of test_gpu_env.py.
# usage: bash tools/gpu_ab.sh <tag> "<lib> <bench args>" ...   (lib relative to element-crush-gym_amd/build)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
declare -A GATED
i=0
for spec in "$@"; do
  set -- $spec
  L=$1; shift
  i=$((i+1))
  export M3_LIB=$PWD/element-crush-gym_amd/build/$L
  if [ -z "${GATED[$L]}" ]; then
    if [ "$FAST" = 1 ]; then
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_checkpoint.py -m gpu -x -q \
        --timeout 300 --timeout-method thread > $OUT/parity_$L.log 2>&1 &&
      timeout -k 10 300 python3 -u -m pytest tests/test_gpu_env.py -m gpu -x -q -k "9x9x6 or 16x16x8" \
        --timeout 300 --timeout-method thread >> $OUT/parity_$L.log 2>&1
    else
      timeout -k 10 600 python3 -u -m pytest ${PARITY_TESTS:-tests/test_gpu_parity.py tests/test_gpu_env.py} -m gpu -x -q \
        --timeout 300 --timeout-method thread > $OUT/parity_$L.log 2>&1
    fi
    rc=$?
    if [ $rc -ge 124 ]; then echo "$L: parity run killed/timed out (rc=$rc)"; exit 1; fi
    GATED[$L]=$rc
  fi
  if [ "${GATED[$L]}" != 0 ]; then echo "$L: REJECTED (parity suite failed, $OUT/parity_$L.log)"; continue; fi
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 64 "$@" > $OUT/$i.log 2>&1 || { tail -5 $OUT/$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$L $*: %.4g env-steps/s  %.3f ms/step  k_env_step %.3f ms  pipeline %.3f ms  oracle_match %s'%(d['value'],d['ms_per_step'],r['hbm']['avg_kernel_ms'],r['pipeline']['avg_ms'],d['parity'].get('oracle_match')))"
done
