set -o pipefail
cd $GRAFT_REPO_ROOT
STZS_LIB=$PWD/tools/variants/libstzs_attn_old.so OUT=gpurun_out/attn_old.json timeout -k 10 120 python -u tools/attn_ab.py > gpurun_out/r06t_attn_old.log 2>&1 && \
OUT=gpurun_out/attn_new.json timeout -k 10 120 python -u tools/attn_ab.py > gpurun_out/r06t_attn_new.log 2>&1 && \
STZS_LIB=$PWD/tools/variants/libstzs_attn_old.so OUT=gpurun_out/attn_old2.json timeout -k 10 120 python -u tools/attn_ab.py > gpurun_out/r06t_attn_old2.log 2>&1 && \
python tools/attn_ab.py --compare gpurun_out/attn_old.json gpurun_out/attn_new.json > gpurun_out/r06t_attn_cmp.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "attention" tests/test_gpu_precise.py > gpurun_out/r06t_tests.log 2>&1
