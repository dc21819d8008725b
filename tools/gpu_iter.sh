# kernel parity tests (GEMM, attention, layers) then the GEMM tile/split sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m pytest tests/test_gemm_gpu.py tests/test_layers_gpu.py tests/test_attention_gpu.py -q -x > gpurun_out/pt_iter.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_iter.log; exit 1; }
tail -2 gpurun_out/pt_iter.log
timeout -k 10 400 python tools/tune_gemm.py tools/step_shapes_c1.json ${TOP:-9} > gpurun_out/tune_iter.log 2>&1 || { echo "tune failed"; tail -5 gpurun_out/tune_iter.log; exit 1; }
echo tune ok
