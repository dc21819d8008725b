# round-4 GPU pass M: forward GEMMs with cold weights / warm activations (the step's cache state)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== cold A/B $(date +%T)"
timeout -k 10 600 python -u tools/ab_cold.py --iters 12 --variants 0,24,26,5,6,7 > gpurun_out/ab_cold.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_cold.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_cold.log
echo "done $(date +%T)"
