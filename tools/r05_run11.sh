cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest11.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05_pytest11.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 120 python3 tools/single_frame.py --calls 300 >> gpurun_out/r05_single11.log 2>&1 || exit 1
  timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt desc_first=0 >> gpurun_out/r05_single11.log 2>&1 || exit 1
done
grep frames_per_call gpurun_out/r05_single11.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench11.log 2>&1
rc=$?; echo "bench rc=$rc"
