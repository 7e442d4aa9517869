cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_detect 16 > gpurun_out/r05_ubench_detect.log 2>&1
rc=$?; echo "ubench_detect rc=$rc"; cat gpurun_out/r05_ubench_detect.log
[ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r05_pytest1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench1.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r05_bench1.log
exit $rc
