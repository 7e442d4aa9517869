cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest37.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest37.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke37.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r05_smoke37.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench37.log 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/r05_bench37.log | cut -c1-400
