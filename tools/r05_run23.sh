cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest23.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest23.log
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/single_frame.py --calls 300 >> gpurun_out/r05_single23.log 2>&1 || exit 1
done
grep frames_per_call gpurun_out/r05_single23.log
rm -rf gpurun_out/single23
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single23 -o run --output-format csv -- python3 tools/single_frame.py --calls 30 > gpurun_out/r05_single23_trace.log 2>&1 || exit 1
echo "trace ok"
