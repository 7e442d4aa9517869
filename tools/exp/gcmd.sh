cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "pyramid" > gpurun_out/t_pyr.log 2>&1; rc=$?; tail -15 gpurun_out/t_pyr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -5 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/b_fused.log 2>&1 || exit 1
SIFT_MI_FUSED_OCTAVE=0 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/b_unfused.log 2>&1 || exit 1
python - <<'PY'
import json
for f in ("b_fused","b_unfused"):
    l=[x for x in open("gpurun_out/%s.log"%f) if x.startswith("{")][-1]
    d=json.loads(l); print(f, round(d["value"]/1e6,2), "Mkp/s", round(d["ms_per_step"],2), "ms", {k:round(v,2) for k,v in d["stage_ms_per_step"].items()}, d["roofline"]["achieved"], d["roofline"]["frac"])
PY
