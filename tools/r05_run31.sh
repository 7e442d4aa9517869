cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for r in 1 2; do
  for v in w1 w5; do
    echo "== $v" >> gpurun_out/r05_ubd31.log
    timeout -k 10 120 ./tools/ubench_detect_$v 64 >> gpurun_out/r05_ubd31.log 2>&1 || exit 1
  done
done
grep -E "==|k_blur_detect  " gpurun_out/r05_ubd31.log
