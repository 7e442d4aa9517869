cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest13.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest13.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for x in 1 0; do
    timeout -k 10 120 python3 tools/single_frame.py --frames 128 --calls 15 --opt xcd_local=$x >> gpurun_out/r05_xcd13.log 2>&1 || exit 1
    timeout -k 10 120 python3 tools/single_frame.py --width 640 --height 480 --frames 256 --calls 20 --opt xcd_local=$x >> gpurun_out/r05_xcd13.log 2>&1 || exit 1
  done
done
grep frames_per_call gpurun_out/r05_xcd13.log
