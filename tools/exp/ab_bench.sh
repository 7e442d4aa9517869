#!/bin/bash
# A/B of env variants on the default bench (no configs / cpu baseline) and the
# single-frame probe.  usage: bash tools/exp/ab_bench.sh "TAG1:ENV=.. ENV2=..[|bench args]" "TAG2:..." ...
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/ab
for spec in "$@"; do
  tag=${spec%%:*}; rest=${spec#*:}; envs=${rest%%|*}; args=""
  [[ $rest == *"|"* ]] && args=${rest#*|}
  env $envs timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-configs $args > gpurun_out/ab/$tag.log 2>&1 || { echo "$tag bench failed"; exit 1; }
  [ -n "$NO_SINGLE" ] && continue
  env $envs TAG=$tag timeout -k 10 120 python tools/exp/single.py >> gpurun_out/ab/single.log 2>&1 || { echo "$tag single failed"; exit 1; }
done
python3 tools/exp/bench_cmp.py gpurun_out/ab/*.log
[ -f gpurun_out/ab/single.log ] && cat gpurun_out/ab/single.log
exit 0
