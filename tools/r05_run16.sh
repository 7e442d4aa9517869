cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for ts in 1 0; do
    timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt tail_split=$ts >> gpurun_out/r05_single16.log 2>&1 || exit 1
  done
done
grep frames_per_call gpurun_out/r05_single16.log
rm -rf gpurun_out/single16
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single16 -o run --output-format csv -- python3 tools/single_frame.py --calls 30 --opt tail_split=0 > gpurun_out/r05_single16_trace.log 2>&1
echo "trace rc=$?"
