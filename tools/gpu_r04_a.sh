set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== v11 tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gemm_v11_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_v11.log 2>&1 || { echo "v11 tests failed"; tail -40 gpurun_out/t_v11.log; exit 1; }
tail -2 gpurun_out/t_v11.log
echo "== ab $(date +%T)"
timeout -k 10 240 python -u tools/ab_v11.py --rounds 4 > gpurun_out/ab_v11.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_v11.log; exit 1; }
grep -v "^{" gpurun_out/ab_v11.log | cut -c1-200
echo "== step parity $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_kd_step_gpu.py -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "training_step" > gpurun_out/t_step.log 2>&1; rc=$?
tail -25 gpurun_out/t_step.log | cut -c1-400
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step tests rc=$rc"; exit 1; fi
echo "== parity report $(date +%T)"
timeout -k 10 400 python -u tools/parity_report.py --out gpurun_out/parity.json > gpurun_out/parity.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/parity.log; exit 1; }
echo "done $(date +%T)"
