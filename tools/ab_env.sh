#!/bin/bash
# Whole-bench A/B of an environment knob (run via gpurun): alternating runs of
# `bench.py --steps 10 --no-configs --no-cpu-baseline` with and without
#   $1 (e.g. SIFT_MI_FUSED_DETECT=0), $2 pairs (default 2); prints value,
# ms_per_step and stage_ms_per_step of each run.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
KV=$1; N=${2:-2}; shift 2
for i in $(seq 1 $N); do
  for mode in base alt; do
    if [ $mode = alt ]; then E="env $KV"; else E=""; fi
    timeout -k 10 300 $E python3 bench.py --steps 10 --warmup 2 --no-configs --no-cpu-baseline --no-latency "$@" > gpurun_out/ab_$mode$i.log 2>&1 || exit 1
    python3 -c "
import json,sys
d=[json.loads(l) for l in open('gpurun_out/ab_$mode$i.log') if l.startswith('{')][0]
s=d['stage_ms_per_step']
print('$mode', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', {k:round(v,3) for k,v in s.items()}, 'frac', round(d['roofline']['frac'],3))"
  done
done
