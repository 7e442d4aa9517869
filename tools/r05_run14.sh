cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_detect_d2 64 > gpurun_out/r05_ubd15.log 2>&1
rc=$?; echo "ubench rc=$rc"; head -8 gpurun_out/r05_ubd15.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_bands.py tests/test_gpu_large.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest15.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest15.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-configs > gpurun_out/r05_bench15.log 2>&1
rc=$?; echo "bench rc=$rc"
