#!/bin/bash
# first GPU validation run: parity tests, short bench, rocprof kernel stats
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --frames 32 --cpu-seconds 6 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run1 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --frames 32 --no-cpu-baseline --no-latency > gpurun_out/prof.log 2>&1
echo "rocprof rc=$?"
find gpurun_out/prof -name "*stats*" | head
