cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in d2 d3 rs; do
  timeout -k 10 120 ./tools/ubench_detect_$v 64 > gpurun_out/r05_ubd5_$v.log 2>&1
  rc=$?; echo "ubench_detect_$v rc=$rc"; cat gpurun_out/r05_ubd5_$v.log
  [ $rc -eq 0 ] || exit $rc
done
# SQ counters of the detection kernels and the octave-0 head kernels, one pass per group
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
SQ2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for grp in "$SQ1" "$SQ2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmc_ubd_$i -o run --output-format csv -- ./tools/ubench_detect_d2 64 > gpurun_out/pmc_ubd_$i.log 2>&1
  rc=$?; echo "pmc ubd $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmc_head_$i -o run --output-format csv -- ./tools/ubench_kernels head 64 > gpurun_out/pmc_head_$i.log 2>&1
  rc=$?; echo "pmc head $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash tools/round_profile.sh r05b 128 trace,fetch,write,sq1,sq2 || exit 1
bash tools/round_profile.sh r05_vga 256 trace,fetch,write,sq1,sq2 640 480 || exit 1
timeout -k 10 300 python tools/bench_bands.py > gpurun_out/r05_bench_bands.log 2>&1
rc=$?; echo "bands rc=$rc"; tail -20 gpurun_out/r05_bench_bands.log
