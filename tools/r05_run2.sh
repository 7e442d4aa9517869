cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in old u1 u3; do
  timeout -k 10 120 ./tools/ubench_detect_$v 64 > gpurun_out/r05_ubd_$v.log 2>&1
  rc=$?; echo "ubench_detect_$v rc=$rc"; cat gpurun_out/r05_ubd_$v.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05_pytest2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline > gpurun_out/r05_bench2.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r05_bench2.log
exit $rc
