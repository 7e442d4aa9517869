#!/bin/bash
# GPU validation run (used via gpurun): parity tests, kernel micro-benchmarks,
# a short bench, and a rocprofv3 kernel-trace profile.  Every GPU step has its
# own time limit; a crash / fault / timeout ends the script.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${1:-tests,ubench,bench,prof}
FRAMES=${FRAMES:-32}
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
if [[ ,$STEPS, == *,tests,* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
if [[ ,$STEPS, == *,ubench,* ]]; then
  timeout -k 10 300 ./tools/ubench_kernels > gpurun_out/ubench.log 2>&1 && timeout -k 10 120 ./tools/ubench_lds >> gpurun_out/ubench.log 2>&1
  rc=$?; echo "ubench rc=$rc"; cat gpurun_out/ubench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ ,$STEPS, == *,blur,* ]]; then
  timeout -k 10 120 ./tools/ubench_kernels blur > gpurun_out/ubench_blur.log 2>&1
  rc=$?; echo "ubench blur rc=$rc"; cat gpurun_out/ubench_blur.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ ,$STEPS, == *,bench,* ]]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --frames $FRAMES --cpu-seconds 6 > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ ,$STEPS, == *,prof,* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --frames $FRAMES --no-cpu-baseline --no-latency > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
