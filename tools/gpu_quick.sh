# GEMM tests, bench line, serialized kernel-trace profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_quick.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_quick.log; exit 1; }
tail -1 gpurun_out/pt_quick.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --serial --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
echo done
