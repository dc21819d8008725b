set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_gemm.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pt_gemm.log; exit 1; }
tail -2 gpurun_out/pt_gemm.log
timeout -k 10 120 python tools/stamp_gemm.py 6144 37888 3584 nt
timeout -k 10 400 python tools/cmp_blas.py ${SHAPES:-tools/step_shapes_c1.json} ${TOP:-24} > gpurun_out/cmp_blas.log 2>&1 || { echo "cmp failed"; tail -20 gpurun_out/cmp_blas.log; exit 1; }
cat gpurun_out/cmp_blas.log
