# round 4 evidence: smoke, the -m gpu suite, bench lines + kernel traces + PMC passes per shape
# (tools/gpu_final.sh), then the batch-1 facade latency
bash tools/gpu_final.sh r04 && timeout -k 10 300 python3 tools/latency.py --out gpurun_out/r04/latency.json > gpurun_out/r04/latency.log 2>&1
