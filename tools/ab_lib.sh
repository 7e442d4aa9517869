#!/bin/bash
# Whole-bench A/B of two builds of libsift_mi.so (run via gpurun): `bash
# tools/ab_lib.sh REPS path/to/alt.so` alternates the product library and the
# alternative (copied over it on the box) REPS times; value, ms/step, stages.
cd "$GRAFT_REPO_ROOT" || exit 2
set -o pipefail
mkdir -p gpurun_out
REPS=$1; ALT=$2
cp sift-features_amd/libsift_mi.so gpurun_out/lib_base.so
for rep in $(seq 1 $REPS); do for v in base alt; do
  if [ $v = base ]; then cp gpurun_out/lib_base.so sift-features_amd/libsift_mi.so; else cp "$ALT" sift-features_amd/libsift_mi.so; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-configs --no-cpu-baseline --no-latency --no-unfused --no-jpeg > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][0]
s=d['stage_ms_per_step']
print('$v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', {k:round(v,3) for k,v in s.items()}, 'frac', round(d['roofline']['frac'],3))"
done; done
cp gpurun_out/lib_base.so sift-features_amd/libsift_mi.so
rm -f gpurun_out/lib_base.so
