# round 4: suite on the 8-configuration library (wide frame, SGPR-spill fix), then the fused-continuation A/B
bash tools/gpu_check.sh r04g libm3_nofuse.so libm3_r03.so && timeout -k 10 300 python3 tools/latency.py --out gpurun_out/r04g/latency.json > gpurun_out/r04g/latency.log 2>&1 && python3 -c "
import json; d=json.load(open('gpurun_out/r04g/latency.json'))
for k,v in d['results'].items(): print(k, round(v['median_us'],1))
print(d['vs_reference'])"
