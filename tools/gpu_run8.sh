set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|passed|failed" gpurun_out/pytest_gpu.log | head -30; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for v in 1 0 1; do
  echo "== bench c1 KD_FUSE_QKV=$v $(date +%T)"
  KD_FUSE_QKV=$v timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-delta > gpurun_out/bench_qkv$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_qkv$v.log; exit 1; }
  tail -1 gpurun_out/bench_qkv$v.log | cut -c1-200
done
