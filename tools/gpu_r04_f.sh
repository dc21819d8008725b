# round-4 GPU pass F: v12 without odd-step barriers (variant 27): bit-exactness, A/B vs v8 (24) and v12 (26)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== v12 tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gemm_v12_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_v12.log 2>&1 || { echo "v12 tests failed"; tail -40 gpurun_out/t_v12.log; exit 1; }
tail -2 gpurun_out/t_v12.log
echo "== ab $(date +%T)"
timeout -k 10 400 python -u tools/ab_v11.py --rounds 4 --variants 24,26,27 > gpurun_out/ab_v12nb.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_v12nb.log; exit 1; }
grep -v "^{" gpurun_out/ab_v12nb.log | cut -c1-250
echo "done $(date +%T)"
