# GPU pass for the parity work (run under gpurun): the whole -m gpu suite, then the
# per-group parity report for the kinds in $PARITY_KINDS.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== tests $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "== parity $(date +%T)"
timeout -k 10 600 python -u tools/parity_report.py --out gpurun_out/parity.json $PARITY_KINDS > gpurun_out/parity.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/parity.log; exit 1; }
echo "done $(date +%T)"
