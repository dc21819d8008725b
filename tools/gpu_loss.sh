# KD-loss parity tests, per-kernel times of the loss on the bench's shape, then the bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kd_loss_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_loss.log 2>&1 || { echo "loss tests failed"; tail -30 gpurun_out/pt_loss.log; exit 1; }
tail -1 gpurun_out/pt_loss.log
rm -rf gpurun_out/bl
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bl -o k -- python3 tools/bench_loss.py 4 loca > gpurun_out/bl.log 2>&1 || { echo "bench_loss failed"; tail -20 gpurun_out/bl.log; exit 1; }
python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/bl/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'kd::' in r['Name']: print(r['Name'][:50], r['Calls'], r['AverageNs'])
"
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-timer > gpurun_out/b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | cut -c1-200
fi
