cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02_pytest1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r02_pytest1.log
[ $rc -eq 0 ] || exit $rc
PMC_OUT=gpurun_out/pmc_r02a bash tools/pmc_bench.sh 'k_seed|k_blur' 128
