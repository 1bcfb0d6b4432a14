set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
{ timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; } && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
