cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/round_profile.sh r05 128 trace,fetch,write,sq1,sq2 || exit 1
bash tools/round_profile.sh r05_vga 256 trace,fetch,write,sq1,sq2 640 480 || exit 1
rm -rf gpurun_out/single
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single -o run --output-format csv -- python3 tools/single_frame.py --calls 30 > gpurun_out/r05_single_trace.log 2>&1
rc=$?; echo "single rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_bands.py > gpurun_out/r05_bench_bands.log 2>&1
rc=$?; echo "bands rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_bands.py --gloo-from /tmp/sift_bands_parts >> gpurun_out/r05_bench_bands.log 2>&1
rc=$?; echo "gloo rc=$rc"; tail -3 gpurun_out/r05_bench_bands.log
du -sh gpurun_out
