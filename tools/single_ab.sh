#!/bin/bash
# one-frame latency A/B over path options (run via gpurun):
#   bash tools/single_ab.sh REPS opt=v [opt=v ...]   ("none=0": the defaults)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
REPS=$1; shift
for rep in $(seq 1 $REPS); do for o in "$@"; do
  if [ "$o" = none=0 ]; then OPT=""; else OPT="--opt $o"; fi
  timeout -k 10 120 python3 tools/single_frame.py --calls 60 $OPT > gpurun_out/single_$o.log 2>&1 || { tail -5 gpurun_out/single_$o.log; exit 1; }
  echo "$o $(grep '^{' gpurun_out/single_$o.log)"
done; done
