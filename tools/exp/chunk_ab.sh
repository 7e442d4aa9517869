#!/bin/bash
# bench.py at several pipeline chunk sizes (GPU box)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --chunk $c --no-cpu-baseline --no-latency > gpurun_out/chunk_$c.log 2>&1 || exit 1
  python3 - "$c" <<'PY'
import json, sys
l = [x for x in open("gpurun_out/chunk_%s.log" % sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print("chunk", sys.argv[1], round(d["value"] / 1e6, 2), "Mkp/s", round(d["ms_per_step"], 2), "ms/step",
      {k: round(v, 2) for k, v in d["stage_ms_per_step"].items()})
PY
done
