set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m pytest tests/test_gemm_gpu.py tests/test_attention_gpu.py -q -x > gpurun_out/pytest_k.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -2 gpurun_out/pytest_k.log
timeout -k 10 200 python tools/bench_attn.py > gpurun_out/bench_attn.log 2>&1 || { echo "bench_attn failed"; tail -20 gpurun_out/bench_attn.log; exit 1; }
cat gpurun_out/bench_attn.log
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || { echo "bench_gemm failed"; tail -20 gpurun_out/bench_gemm.log; exit 1; }
cat gpurun_out/bench_gemm.log
