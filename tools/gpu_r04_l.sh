# round-4 GPU pass L: q|k|v scatter epilogue A/B across GEMM builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== qkv A/B $(date +%T)"
timeout -k 10 300 python -u tools/ab_qkv.py --rounds 4 > gpurun_out/ab_qkv.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_qkv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_qkv.log
echo "done $(date +%T)"
