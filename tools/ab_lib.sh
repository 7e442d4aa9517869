#!/bin/bash
# Whole-bench A/B of the product library and an alternative build of it (run
# via gpurun): `bash tools/ab_lib.sh REPS path/to/alt.so` alternates the two
# REPS times (the alternative through SIFT_MI_LIB, sift-features_amd/_lib.py)
# and prints value, ms/step and stage times per run.
cd "$GRAFT_REPO_ROOT" || exit 2
set -o pipefail
mkdir -p gpurun_out
REPS=$1; ALT=$2
for rep in $(seq 1 $REPS); do for v in base alt; do
  if [ $v = base ]; then unset SIFT_MI_LIB; else export SIFT_MI_LIB="$ALT"; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-configs --no-cpu-baseline --no-latency --no-unfused --no-jpeg > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][0]
s=d['stage_ms_per_step']
print('$v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', {k:round(v,3) for k,v in s.items()}, 'frac', round(d['roofline']['frac'],3))"
done; done
