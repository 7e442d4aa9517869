# round-6 GPU A/B driver (run via gpurun): pair-kernel micro-benchmark at two
# wave targets, then whole-bench pairs over the path options given as args
set -o pipefail
mkdir -p gpurun_out
for w in 8192 4096; do BD_WAVES=$w timeout -k 10 60 tools/ubench_detect 64 > gpurun_out/ubd_$w.log 2>&1 || { cat gpurun_out/ubd_$w.log; exit 1; }; grep -E "k_blur_detect" gpurun_out/ubd_$w.log; done
for rep in 1 2; do for o in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-configs --no-cpu-baseline --no-latency --no-unfused --no-jpeg --opt $o > gpurun_out/ab_$o.log 2>&1 || exit 1
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_$o.log') if l.startswith('{')][0]
s=d['stage_ms_per_step']
print('$o', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', {k:round(v,3) for k,v in s.items()}, 'frac', round(d['roofline']['frac'],3))"
done; done
