# input-pipeline parity tests (depth transform + image preprocessing) and their timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_depth.py tests/test_image.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_pre.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pt_pre.log; exit 1; }
tail -2 gpurun_out/pt_pre.log
timeout -k 10 200 python -u tools/bench_image.py > gpurun_out/bench_image.log 2>&1 || { echo "bench_image failed"; tail -20 gpurun_out/bench_image.log; exit 1; }
cat gpurun_out/bench_image.log
echo done
