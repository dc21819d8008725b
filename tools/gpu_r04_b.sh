# round-4 GPU pass B: the wide-row DMA diagnostic (variant 25) vs v8 (24) and v11 (23)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== ab $(date +%T)"
timeout -k 10 300 python -u tools/ab_v11.py --rounds 4 --variants 24,25,23 > gpurun_out/ab_wide.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_wide.log; exit 1; }
grep -v "^{" gpurun_out/ab_wide.log | cut -c1-250
echo "done $(date +%T)"
