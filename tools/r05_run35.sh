cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for d in 2 0; do
    timeout -k 10 120 python3 tools/single_frame.py --calls 20 --frames 128 --opt onesweep=$d >> gpurun_out/r05_batch35.log 2>&1 || exit 1
    timeout -k 10 120 python3 tools/single_frame.py --calls 30 --frames 256 --width 640 --height 480 --opt onesweep=$d >> gpurun_out/r05_vga35.log 2>&1 || exit 1
  done
done
grep -h frames_per_call gpurun_out/r05_batch35.log gpurun_out/r05_vga35.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l[l.index('{'):]); print(d['frame'], d['path_options'], round(d['ms_per_call_median'],3))"
