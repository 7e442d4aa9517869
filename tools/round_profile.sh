#!/bin/bash
# Round profile (run via gpurun): the bench command under rocprofv3
# --kernel-trace --stats, then two separate PMC passes (FETCH_SIZE, WRITE_SIZE;
# no trace domains mixed with --pmc) over the same command, summarised into
# profiles/<round>_* by tools/profile_summary.py.
#   bash tools/round_profile.sh r01 [frames]   (default: bench.py's 128 frames per call)
cd "$GRAFT_REPO_ROOT" || exit 2
ROUND=${1:-r01}
FRAMES=${2:-128}
OUT=gpurun_out/rp_$ROUND
rm -rf "$OUT"
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --steps 3 --warmup 1 --frames $FRAMES --no-cpu-baseline --no-latency"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $CMD > $OUT/bench_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $CMD > $OUT/bench_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
# summarise locally after gpurun merges gpurun_out/ back:
#   python3 tools/profile_summary.py $ROUND $OUT $FRAMES
python3 tools/profile_summary.py $ROUND $OUT $FRAMES > $OUT/summary.md
