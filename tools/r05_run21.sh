cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest21.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest21.log
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for d in 0 1; do
    timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt sync_scope=$d >> gpurun_out/r05_single21.log 2>&1 || exit 1
  done
done
grep frames_per_call gpurun_out/r05_single21.log
rm -rf gpurun_out/single21
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single21 -o run --output-format csv -- python3 tools/single_frame.py --calls 30 > gpurun_out/r05_single21_trace.log 2>&1 || exit 1
echo "trace ok"
timeout -k 10 300 python3 bench.py > gpurun_out/r05_bench21.log 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/r05_bench21.log | cut -c1-600
