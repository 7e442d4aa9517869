#!/bin/bash
# k_octave investigation: kernel trace of a 1-step bench + PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/octtr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/octtr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --frames 32 --no-cpu-baseline --no-latency > gpurun_out/octtr.log 2>&1 || exit 1
bash tools/pmc_bench.sh k_octave 32 || exit 1
python3 tools/pmc_summary.py k_octave gpurun_out/pmcb/p*/*/*counter_collection.csv > gpurun_out/oct_pmc.txt 2>&1 || python3 tools/pmc_summary.py k_octave $(find gpurun_out/pmcb -name "*counter_collection.csv") > gpurun_out/oct_pmc.txt
cat gpurun_out/oct_pmc.txt
