cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for r in 1 2; do
for v in s256b0 s256b1 s384b1 s512b1; do
  timeout -k 10 120 ./tools/ubench_detect_$v 64 > gpurun_out/r05_ubd10_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(grep -E 'k_blur_detect  |G_5' gpurun_out/r05_ubd10_$v.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_extensions.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest10.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05_pytest10.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 120 python3 tools/single_frame.py --calls 300 >> gpurun_out/r05_single10.log 2>&1 || exit 1
  timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt desc_first=0 >> gpurun_out/r05_single10.log 2>&1 || exit 1
done
grep frames_per_call gpurun_out/r05_single10.log
