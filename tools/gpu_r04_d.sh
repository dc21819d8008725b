# round-4 GPU pass D: smoke(), the whole -m gpu suite, attention timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== attn $(date +%T)"
timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/bench_attn.log 2>&1 || { echo "attn bench failed"; tail -10 gpurun_out/bench_attn.log; exit 1; }
cat gpurun_out/bench_attn.log | grep -v amdgpu.ids
echo "== tests $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc $(date +%T)"
