# The GPU suite, then the descriptor ablation micro-benchmark (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 tools/ubench_kernels desc > gpurun_out/ubk_desc.log 2>&1 || exit 1
cat gpurun_out/ubk_desc.log
