#!/bin/bash
# Round evidence (run via gpurun): the default bench line, then the round
# profile (trace + PMC passes) of the same workload
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/r06_bench.log 2>&1 || { tail -20 gpurun_out/r06_bench.log; exit 1; }
grep '^{' gpurun_out/r06_bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.readline())
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'stages', d['stage_ms_per_step'])
print('latency', d.get('latency_1frame_ms'), 'cpu', d['cpu_baseline'])
print('configs', json.dumps(d.get('configs'))[:1500])"
bash tools/round_profile.sh ${1:-r06} 128 || exit 1
head -12 gpurun_out/rp_${1:-r06}/summary.md
