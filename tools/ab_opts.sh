#!/bin/bash
# Whole-bench A/B over path options (run via gpurun): `bash tools/ab_opts.sh
# REPS opt=v [opt=v ...]` alternates `bench.py --steps 10 --opt <each>` REPS
# times on one box and prints value, ms/step, stage times and frac per run
# (use "none=0" for the product defaults, "chunk=K" for --chunk K; EXTRA: more
# bench.py arguments, e.g. EXTRA="--frames 256 --width 640 --height 480").
cd "$GRAFT_REPO_ROOT" || exit 2
set -o pipefail
mkdir -p gpurun_out
REPS=$1; shift
for rep in $(seq 1 $REPS); do for o in "$@"; do
  case $o in none=0) OPT="";; chunk=*) OPT="--chunk ${o#chunk=}";; *) OPT="--opt $o";; esac
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-configs --no-cpu-baseline --no-latency --no-unfused --no-jpeg $EXTRA $OPT > gpurun_out/ab_$o.log 2>&1 || { tail -5 gpurun_out/ab_$o.log; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_$o.log') if l.startswith('{')][0]
s=d['stage_ms_per_step']
print('$o', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', {k:round(v,3) for k,v in s.items()}, 'frac', round(d['roofline']['frac'],3))"
done; done
