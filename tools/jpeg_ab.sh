#!/bin/bash
# JPEG pipeline A/B (run via gpurun): tools/bench_jpeg.py over host decode
# thread counts (decode-only, serial and pipelined frames/s each).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for t in ${@:-8 12 16}; do
  timeout -k 10 300 python3 tools/bench_jpeg.py --threads $t --steps 4 >> gpurun_out/jpeg_ab.log 2>&1 || exit $?
  tail -1 gpurun_out/jpeg_ab.log
done
