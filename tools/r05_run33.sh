cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest33.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest33.log
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for d in 1 0; do
    timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt onesweep=$d >> gpurun_out/r05_single33.log 2>&1 || exit 1
  done
done
for r in 1 2; do
  for d in 1 0; do
    timeout -k 10 120 python3 tools/single_frame.py --calls 20 --frames 128 --opt onesweep=$d >> gpurun_out/r05_batch33.log 2>&1 || exit 1
  done
done
grep frames_per_call gpurun_out/r05_single33.log gpurun_out/r05_batch33.log
rm -rf gpurun_out/single33
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single33 -o run --output-format csv -- python3 tools/single_frame.py --calls 30 --opt onesweep=1 > gpurun_out/r05_single33_trace.log 2>&1 || exit 1
echo "trace ok"
