#!/bin/bash
# Round-4 measurement call (run via gpurun): the steps named in $1 (comma
# list; default all), each under its own time limit; the first failure ends
# the script.
#   prof   tools/round_profile.sh r04 (1080p x 128: trace + PMC passes)
#   vga    tools/round_profile.sh r04_vga (640x480 x 256: trace + FETCH / WRITE)
#   single rocprofv3 kernel trace of 30 single-frame calls (tools/single_frame.py)
#   jpeg   tools/jpeg_ab.sh (decode threads 8 / 12 / 16)
#   bands  tools/bench_bands.py (8192^2 by row bands)
#   vgachunk  256 x 640x480 per call: auto chunks (2 x 128, two lanes) vs one
#          chunk of 256 (one lane + octave overlap), two pairs
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
S=",${1:-prof,vga,single,jpeg,bands},"
if [[ $S == *,prof,* ]]; then bash tools/round_profile.sh r04 || exit 1; fi
if [[ $S == *,vga,* ]]; then bash tools/round_profile.sh r04_vga 256 trace,fetch,write 640 480 || exit 1; fi
if [[ $S == *,single,* ]]; then
  rm -rf gpurun_out/single
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single -o run --output-format csv -- python3 tools/single_frame.py --calls 30 > gpurun_out/single.log 2>&1
  rc=$?; echo "single rc=$rc"; tail -1 gpurun_out/single.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 tools/single_frame.py --calls 200 >> gpurun_out/single.log 2>&1 || exit 1
  tail -1 gpurun_out/single.log
fi
if [[ $S == *,jpeg,* ]]; then bash tools/jpeg_ab.sh 8 12 16 || exit 1; fi
if [[ $S == *,vgachunk,* ]]; then
  for i in 1 2; do for ch in 0 256; do
    timeout -k 10 300 python3 bench.py --frames 256 --width 640 --height 480 --chunk $ch --steps 10 --no-configs --no-cpu-baseline --no-latency > gpurun_out/vga_ch$ch.log 2>&1 || exit 1
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/vga_ch$ch.log') if l.startswith('{')][0]
print('vga chunk $ch', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms frac', round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['stage_ms_per_step'].items()})"
  done; done
fi
if [[ $S == *,bands,* ]]; then
  timeout -k 10 300 python3 tools/bench_bands.py > gpurun_out/bench_bands.log 2>&1; rc=$?
  echo "bands rc=$rc"; tail -1 gpurun_out/bench_bands.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
