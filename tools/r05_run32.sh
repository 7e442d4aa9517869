cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest32.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest32.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/stress_paths.py --rounds 2 > gpurun_out/r05_stress32.log 2>&1
rc=$?; echo "stress rc=$rc"; tail -1 gpurun_out/r05_stress32.log
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for d in 1 0; do
    timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt large_first=$d >> gpurun_out/r05_single32.log 2>&1 || exit 1
  done
done
grep frames_per_call gpurun_out/r05_single32.log
for d in 1 0; do
rm -rf gpurun_out/single32_$d
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single32_$d -o run --output-format csv -- python3 tools/single_frame.py --calls 30 --opt large_first=$d > gpurun_out/r05_single32_trace.log 2>&1 || exit 1
done
echo "trace ok"
