# round-4 GPU pass Q: pre-tiled B (bit-exactness, A/B warm and cold)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== pretiled tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gemm_pretiled_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_pretiled.log 2>&1 || { echo "pretiled tests failed"; tail -40 gpurun_out/t_pretiled.log; exit 1; }
tail -2 gpurun_out/t_pretiled.log
echo "== ab $(date +%T)"
timeout -k 10 400 python -u tools/ab_pretiled.py --iters 10 > gpurun_out/ab_pretiled.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_pretiled.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_pretiled.log
echo "done $(date +%T)"
