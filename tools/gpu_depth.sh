# depth-transform parity tests + kernel timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_depth.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_depth.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pt_depth.log; exit 1; }
tail -2 gpurun_out/pt_depth.log
timeout -k 10 200 python -u tools/bench_depth.py > gpurun_out/bench_depth.log 2>&1 || { echo "bench_depth failed"; tail -20 gpurun_out/bench_depth.log; exit 1; }
cat gpurun_out/bench_depth.log
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_depth -o run -- python3 tools/bench_depth.py > gpurun_out/prof_depth.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_depth.log; exit 1; }
fi
echo done
