#!/bin/bash
# Round profile (run via gpurun): the bench command under rocprofv3
# --kernel-trace --stats, then separate PMC passes (FETCH_SIZE; WRITE_SIZE; two
# SQ groups -- no trace domains mixed with --pmc) over the same command,
# summarised into profiles/<round>_* by tools/profile_summary.py.
#   bash tools/round_profile.sh r04 [frames] [passes] [W] [H]
#   (default: bench.py's 128 frames per call at 1920x1080)
cd "$GRAFT_REPO_ROOT" || exit 2
ROUND=${1:-r04}
FRAMES=${2:-128}
PASSES=",${3:-trace,fetch,write,sq1,sq2},"
W=${4:-1920}
H=${5:-1080}
OUT=gpurun_out/rp_$ROUND
mkdir -p "$OUT"
export TMPDIR=/tmp
# the default bench workload only: no CPU baseline, no latency probe, no
# other-config runs (they would mix other frame sizes into the PMC means)
CMD="python3 bench.py --steps 3 --warmup 1 --frames $FRAMES --width $W --height $H --no-cpu-baseline --no-latency --no-configs --no-unfused"
pass() {  # name, rocprofv3 options
  local name=$1; shift
  rm -rf "$OUT/$name"
  timeout -k 10 600 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- $CMD > $OUT/bench_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
if [[ $PASSES == *,trace,* ]]; then pass trace --kernel-trace --stats || exit 1; fi
if [[ $PASSES == *,fetch,* ]]; then pass fetch --pmc FETCH_SIZE || exit 1; fi
if [[ $PASSES == *,write,* ]]; then pass write --pmc WRITE_SIZE || exit 1; fi
if [[ $PASSES == *,sq1,* ]]; then
  pass sq1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU || exit 1
fi
if [[ $PASSES == *,sq2,* ]]; then
  pass sq2 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE || exit 1
fi
python3 tools/profile_summary.py $ROUND $OUT $FRAMES $W $H > $OUT/summary.md
# keep gpurun_out/ under gpurun's 64 MiB merge limit: compress the raw CSVs
find $OUT -name '*.csv' -size +256k -exec gzip -9 {} \;
du -sh $OUT
