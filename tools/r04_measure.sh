#!/bin/bash
# Round-4 measurement call (run via gpurun): the steps named in $1 (comma
# list; default all), each under its own time limit; the first failure ends
# the script.
#   prof   tools/round_profile.sh r04 (1080p x 128: trace + PMC passes)
#   vga    tools/round_profile.sh r04_vga (640x480 x 256: trace + FETCH / WRITE)
#   single rocprofv3 kernel trace of 30 single-frame calls (tools/single_frame.py)
#   jpeg   tools/jpeg_ab.sh (decode threads 8 / 12 / 16)
#   bands  tools/bench_bands.py (8192^2 by row bands)
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
if [[ $S == *,bands,* ]]; then
  timeout -k 10 300 python3 tools/bench_bands.py > gpurun_out/bench_bands.log 2>&1; rc=$?
  echo "bands rc=$rc"; tail -1 gpurun_out/bench_bands.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
