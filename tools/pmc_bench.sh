#!/bin/bash
# PMC counter passes over a short bench run, restricted to kernels matching $1
# (one counter group per pass; no trace domains mixed with --pmc).
#   bash tools/pmc_bench.sh <kernel-regex> [frames]
cd "$GRAFT_REPO_ROOT" || exit 2
RE=${1:-k_detect}
FRAMES=${2:-32}
OUT=${PMC_OUT:-gpurun_out/pmcb}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --steps 1 --warmup 0 --frames $FRAMES --no-cpu-baseline --no-latency"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp --kernel-include-regex "$RE" -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
