set -o pipefail
cd $GRAFT_REPO_ROOT
OLD=$PWD/tools/variants/wt/styletts-zs_amd/stzs/libstzs_hip.so
STZS_LIB=$OLD timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06u_hash_old.txt 2> gpurun_out/r06u_hash_old.err && \
timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06u_hash_new.txt 2> gpurun_out/r06u_hash_new.err && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lnrows.py tests/test_gpu_ops.py tests/test_gpu_fp8.py tests/test_gpu_rows.py > gpurun_out/r06u_tests.log 2>&1
