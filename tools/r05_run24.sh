cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rank.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest24.log 2>&1
echo "rank tests rc=$?"; grep -E "passed|failed|assert|Error" gpurun_out/r05_pytest24.log | head -20
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -q -k "paths_equal" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_pytest24b.log 2>&1
echo "paths rc=$?"; grep -E "passed|failed|assert " gpurun_out/r05_pytest24b.log | head -20
