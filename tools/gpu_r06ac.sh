set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06ac_hash.txt 2> gpurun_out/r06ac_hash.err && \
timeout -k 10 300 python -u tools/back_launches.py > gpurun_out/r06ac_back.txt 2> gpurun_out/r06ac_back.err && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_abi_generic.py tests/test_gpu_configs.py > gpurun_out/r06ac_tests.log 2>&1
