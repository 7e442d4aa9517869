set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py > gpurun_out/pytest_fused.log 2>&1 || { tail -30 gpurun_out/pytest_fused.log; exit 1; }
tail -2 gpurun_out/pytest_fused.log
bash tools/gcmd_r06.sh bd_pair=1 bd_pair=2
