cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_detect_d2 64 > gpurun_out/r05_ubd8.log 2>&1
rc=$?; echo "ubench_detect rc=$rc"; head -8 gpurun_out/r05_ubd8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_batch.py tests/test_gpu_bands.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest8.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05_pytest8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench8.log 2>&1
rc=$?; echo "bench rc=$rc"
