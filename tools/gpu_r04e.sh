bash tools/gpu_check.sh r04f libm3_nofuse.so libm3_r03.so libm3_l16.so && timeout -k 10 300 python3 tools/latency.py --out gpurun_out/r04f/latency.json > gpurun_out/r04f/latency.log 2>&1 && M3_LIB=$PWD/element-crush-gym_amd/build/libm3.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04f/kt9 -o kt --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > gpurun_out/r04f/kt9.log 2>&1; python3 -c "
import json; d=json.load(open('gpurun_out/r04f/latency.json'))
for k,v in d['results'].items(): print(k, round(v['median_us'],1))
print(d['vs_reference'])"
