cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest36.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_pytest36.log
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for d in 1 0; do
    timeout -k 10 120 python3 tools/single_frame.py --calls 300 --opt desc_reverse=$d >> gpurun_out/r05_single36.log 2>&1 || exit 1
  done
done
grep -h frames_per_call gpurun_out/r05_single36.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l[l.index('{'):]); print(d['path_options'], round(d['ms_per_call_median'],4), round(d['ms_per_call'],4))"
rm -rf gpurun_out/single36
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single36 -o run --output-format csv -- python3 tools/single_frame.py --calls 30 --opt desc_reverse=1 > gpurun_out/r05_single36_trace.log 2>&1 || exit 1
echo "trace ok"
