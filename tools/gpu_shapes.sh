# per-shape GEMM table of the bench step + kd_gemm vs hipBLASLt on the top shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --shapes gpurun_out/shapes.json > gpurun_out/bench_shapes.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_shapes.log; exit 1; }
tail -1 gpurun_out/bench_shapes.log
timeout -k 10 300 python tools/cmp_blas.py gpurun_out/shapes.json ${TOP:-24} > gpurun_out/cmp_blas.log 2>&1 || { echo "cmp failed"; tail -20 gpurun_out/cmp_blas.log; exit 1; }
cat gpurun_out/cmp_blas.log
