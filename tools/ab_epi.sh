set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_bench_shapes_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_epi.log 2>&1 || { tail -30 gpurun_out/t_epi.log; exit 1; }
tail -2 gpurun_out/t_epi.log
for lib in base new; do
  if [ $lib = base ]; then export KDSTEP_LIB=$PWD/ab/libkdstep_base.so; else unset KDSTEP_LIB; fi
  echo "== $lib"; EPI_SHAPES="siglip o,fc2,0.5b o,0.5b down,7b o,7b down,wgrad" timeout -k 10 300 python tools/epi_cost.py 30 0 || exit 1
done > gpurun_out/ab_epi.log 2>&1
cat gpurun_out/ab_epi.log
for nt in 0 1; do for bl in 16384 2048; do echo "NT=$nt blocks=$bl"; KD_ADAMW_NT=$nt KD_ADAMW_BLOCKS=$bl timeout -k 10 100 python tools/bench_adamw.py || exit 1; done; done > gpurun_out/adamw.log 2>&1; cat gpurun_out/adamw.log
