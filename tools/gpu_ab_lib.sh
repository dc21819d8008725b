# GPU pass for a library A/B (run under gpurun): the whole -m gpu suite on the in-tree library,
# then the c1 bench alternating the in-tree build ("new") and tools/variants/libkdstep_base.so
# ("base", loaded through KDSTEP_LIB), with the fused q|k|v epilogue on and off (KD_FUSE_QKV).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|passed|failed" gpurun_out/pytest_gpu.log | head -30; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in "new 1" "base 1" "new 0" "new 1" "base 1"; do
  set -- $cfg
  if [ $1 = base ]; then export KDSTEP_LIB=$PWD/tools/variants/libkdstep_base.so; else unset KDSTEP_LIB; fi
  echo "== bench c1 lib=$1 KD_FUSE_QKV=$2 $(date +%T)"
  KD_FUSE_QKV=$2 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-delta > gpurun_out/bench_$1_qkv$2.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$1_qkv$2.log; exit 1; }
  tail -1 gpurun_out/bench_$1_qkv$2.log | cut -c1-200
done
