set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "v9 or variants_all or variant_epilogue" > gpurun_out/pt_v9.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_v9.log; exit 1; }
tail -1 gpurun_out/pt_v9.log
KD_VARIANTS=16,20 timeout -k 10 400 python tools/cmp_blas.py tools/step_shapes_c1.json ${TOP:-16} > gpurun_out/cmp_v9.log 2>&1 || { echo "cmp failed"; tail -20 gpurun_out/cmp_v9.log; exit 1; }
cat gpurun_out/cmp_v9.log
