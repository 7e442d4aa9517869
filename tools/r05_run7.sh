cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in d2 pk; do
  timeout -k 10 120 ./tools/ubench_detect_$v 64 > gpurun_out/r05_ubd7_$v.log 2>&1
  rc=$?; echo "ubench_detect_$v rc=$rc"; cat gpurun_out/r05_ubd7_$v.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_batch.py tests/test_gpu_bands.py tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05_pytest7.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-configs > gpurun_out/r05_bench7.log 2>&1
rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
for o in tail_split=1 tail_split=0 fused_detect=3 tail_split=1 tail_split=0 fused_detect=3; do
  timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt $o >> gpurun_out/r05_single7.log 2>&1 || exit 1
done
tail -3 gpurun_out/r05_single7.log
for ts in 1 0 1 0; do
  timeout -k 10 120 python3 tools/single_frame.py --width 640 --height 480 --frames 256 --calls 30 --opt tail_split=$ts >> gpurun_out/r05_vga7.log 2>&1 || exit 1
  timeout -k 10 120 python3 tools/single_frame.py --frames 128 --calls 15 --opt tail_split=$ts >> gpurun_out/r05_b1087.log 2>&1 || exit 1
done
cat gpurun_out/r05_vga7.log gpurun_out/r05_b1087.log | grep frames_per_call
