tail -2 gpurun_out/pytest_gpu.log; grep stamps gpurun_out/stamps.log
for f in gpurun_out/bench_serial.log gpurun_out/bench.log; do grep '^{' $f | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('$f', round(d['value']/1e9,2), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()}, d['roofline']['frac'], d['pipeline_roofline']['frac'])"; done
