cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
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
rm -rf gpurun_out/single
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/single -o run --output-format csv -- python3 tools/single_frame.py --calls 30 > gpurun_out/single.log 2>&1
rc=$?; echo "single rc=$rc"; tail -1 gpurun_out/single.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/single_frame.py --calls 200 >> gpurun_out/single.log 2>&1 || exit 1
tail -1 gpurun_out/single.log
bash tools/round_profile.sh r05b 128 trace,fetch,write,sq1,sq2 || exit 1
bash tools/round_profile.sh r05_vga 256 trace,fetch,write,sq1,sq2 640 480 || exit 1
timeout -k 10 300 python tools/bench_bands.py > gpurun_out/r05_bench_bands.log 2>&1
rc=$?; echo "bands rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_bands.py --gloo-from /tmp/sift_bands_parts >> gpurun_out/r05_bench_bands.log 2>&1
rc=$?; echo "gloo rc=$rc"; tail -5 gpurun_out/r05_bench_bands.log
du -sh gpurun_out
