cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest28.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest28.log
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt graph=$g >> gpurun_out/r05_single28.log 2>&1 || exit 1
  done
done
grep frames_per_call gpurun_out/r05_single28.log
