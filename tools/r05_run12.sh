cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/single12
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single12 -o run --output-format csv -- python3 tools/single_frame.py --calls 30 > gpurun_out/r05_single12_trace.log 2>&1
rc=$?; echo "single rc=$rc"; [ $rc -eq 0 ] || exit $rc
