set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kd_step_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_step.log 2>&1; echo "step tests rc=$?"; tail -15 gpurun_out/pytest_step.log | grep -v "^$"
timeout -k 10 600 python -u tools/parity_report.py --out gpurun_out/parity.json lb dt1 fb bd sun_lb mix_fb > gpurun_out/parity.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/parity.log; exit 1; }
echo "== bench c1 $(date +%T)"
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_c1.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log | cut -c1-400
for f in all lm_mlp; do
  echo "== bench c4 $f $(date +%T)"
  timeout -k 10 600 python -u bench.py --config c4 --fp8-families $f --no-cpu-baseline --no-delta > gpurun_out/bench_c4_$f.log 2>&1 || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4_$f.log; exit 1; }
  tail -1 gpurun_out/bench_c4_$f.log | cut -c1-300
done
