#!/bin/bash
# bench.py under alternative environment settings, e.g.
#   bash tools/exp/env_ab.sh "SIFT_MI_STAGGER=0" "SIFT_MI_STAGGER=1" "SIFT_MI_STAGGER=1 CHUNK=32"
# (CHUNK=n passes --chunk n)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  chunk=0
  for kv in $spec; do case $kv in CHUNK=*) chunk=${kv#CHUNK=};; esac; done
  env $(echo $spec | tr ' ' '\n' | grep -v '^CHUNK=') timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --chunk $chunk --no-cpu-baseline --no-latency > gpurun_out/env_$i.log 2>&1 || exit 1
  python3 - "$i" "$spec" <<'PY'
import json, sys
l = [x for x in open("gpurun_out/env_%s.log" % sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], "|", round(d["value"] / 1e6, 2), "Mkp/s", round(d["ms_per_step"], 2), "ms/step serial", round(d["serial_lane_ms_per_step"], 2))
PY
done
