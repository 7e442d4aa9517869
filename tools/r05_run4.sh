cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ubench_kernels_old ubench_kernels; do
  timeout -k 10 120 ./tools/$v head 64 > gpurun_out/r05_head_$v.log 2>&1
  rc=$?; echo "$v head rc=$rc"; cat gpurun_out/r05_head_$v.log
  [ $rc -eq 0 ] || exit $rc
done
for v in old v2; do
  timeout -k 10 120 ./tools/ubench_detect_$v 64 > gpurun_out/r05_ubd4_$v.log 2>&1
  rc=$?; echo "ubench_detect_$v rc=$rc"; cat gpurun_out/r05_ubd4_$v.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05_pytest4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench4.log 2>&1
rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/round_profile.sh r05a 128 trace
