# Round-end style GPU pass: parity tests, PMC HBM traffic (2 passes), the bench line, and the
# kernel-trace profile of a serialized bench (its forward-GEMM average is what the roofline
# pass of bench.py measures with HIP events)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
if [ "${PMC:-1}" = "1" ]; then
  bash tools/pmc_bench.sh > gpurun_out/pmc_bench.log 2>&1 || { echo "pmc failed"; tail -10 gpurun_out/pmc_bench.log; exit 1; }
  cp gpurun_out/pmc_traffic.json profiles/r01/pmc_traffic.json
fi
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --serial --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
echo done
