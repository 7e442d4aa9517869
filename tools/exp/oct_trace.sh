#!/bin/bash
# Per-octave pyramid kernel durations (GPU box): rocprofv3 kernel trace of a
# 1-step, 32-frame bench, per-blur path and fused path.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
for f in 0 1; do
  rm -rf gpurun_out/otr$f
  SIFT_MI_FUSED_OCTAVE=$f timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/otr$f -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --frames 32 --no-cpu-baseline --no-latency > gpurun_out/otr$f.log 2>&1 || exit 1
done
