#!/bin/bash
# JPEG pipeline A/B (run via gpurun): tools/bench_jpeg.py (decode-only,
# serial and pipelined frames/s) per configuration; a configuration is
# "<threads>[:VAR=value,...]", e.g. 16 16:SIFT_MI_WAIT=spin 16:GPU_MAX_HW_QUEUES=8
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for cfg in ${@:-8 12 16}; do
  t=${cfg%%:*}; envs=""
  [[ $cfg == *:* ]] && envs=$(echo "${cfg#*:}" | tr ',' ' ')
  echo "== threads $t $envs" >> gpurun_out/jpeg_ab.log
  timeout -k 10 300 env $envs python3 tools/bench_jpeg.py --threads $t --steps 4 >> gpurun_out/jpeg_ab.log 2>&1 || exit $?
  echo "$cfg: $(tail -1 gpurun_out/jpeg_ab.log)"
done
