#!/bin/bash
# PMC passes over a kernel micro-benchmark (counters in separate passes; no
# trace domains combined with --pmc).  $1: passes, $2: the binary's argument
# (ubench_kernels: blur | desc; ubench_detect: frames); BIN: the binary.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() { timeout -k 10 300 rocprofv3 --pmc $1 -d gpurun_out/pmc/$2 -o p --output-format csv -- $BIN $MODE > gpurun_out/pmc/$2.log 2>&1; local rc=$?; echo "$2 rc=$rc"; return $rc; }
PASSES=",${1:-sq1,sq2,fetch,write},"
MODE=${2:-blur}
BIN=${BIN:-./tools/ubench_kernels}
timeout -k 10 120 $BIN $MODE > gpurun_out/pmc/timing.log 2>&1 || exit 1
[[ $PASSES == *,sq1,* ]] && { run "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" sq1 || exit 1; }
[[ $PASSES == *,sq2,* ]] && { run "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" sq2 || exit 1; }
[[ $PASSES == *,fetch,* ]] && { run "FETCH_SIZE" fetch || exit 1; }
[[ $PASSES == *,write,* ]] && { run "WRITE_SIZE" write || exit 1; }
exit 0
