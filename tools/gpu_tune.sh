# GEMM parity tests, then the kernel x tile x split-K sweep over the step's GEMM shapes (refits plan_gemm)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_gemm.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pt_gemm.log; exit 1; }
tail -2 gpurun_out/pt_gemm.log
timeout -k 10 600 python tools/tune_gemm.py tools/step_shapes_c1.json ${TOP:-60} > gpurun_out/gemm_tune.jsonl 2> gpurun_out/gemm_tune.err || { echo "tune failed"; tail -20 gpurun_out/gemm_tune.err; exit 1; }
wc -l gpurun_out/gemm_tune.jsonl
