# k_loss_grad geometry sweep: bench_loss under each tools/variants/lg_* library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in tools/variants/lg_*; do
  rm -rf gpurun_out/blv
  KDSTEP_LIB=$PWD/$d/libkdstep.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/blv -o k -- python3 tools/bench_loss.py 4 loca > gpurun_out/blv.log 2>&1 || { echo "$d failed"; tail -5 gpurun_out/blv.log; exit 1; }
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/blv/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'loss_grad' in r['Name']: print('$d', r['Calls'], r['AverageNs'])
"
done
