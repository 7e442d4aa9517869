#!/bin/bash
# bench.py with alternative library builds (tools/exp/v_<name>/libsift_mi.so; "base" = the in-tree one)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then unset SIFT_MI_LIB; else export SIFT_MI_LIB=tools/exp/v_$v/libsift_mi.so; fi
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/lib_$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import json, sys
l = [x for x in open("gpurun_out/lib_%s.log" % sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], round(d["value"] / 1e6, 2), "Mkp/s", round(d["ms_per_step"], 2), "ms/step",
      {k: round(v, 2) for k, v in d["stage_ms_per_step"].items()})
PY
done
