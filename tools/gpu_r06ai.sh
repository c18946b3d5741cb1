set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_bench.sh r06 > gpurun_out/r06ai_pmc.log 2>&1 && \
bash tools/prof.sh prof_r06ai && \
python3 tools/roofline_check.py gpurun_out/prof_r06ai/run_kernel_trace.csv gpurun_out/prof_r06ai.log > gpurun_out/roofline_check_r06ai.json
