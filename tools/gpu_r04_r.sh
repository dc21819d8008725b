# round-4 GPU pass R: prefetching a GEMM's cold weights (kd_prefetch) right before it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== prefetch A/B $(date +%T)"
timeout -k 10 400 python -u tools/ab_cold.py --iters 12 --prefetch > gpurun_out/ab_prefetch.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_prefetch.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_prefetch.log
echo "done $(date +%T)"
echo "== step A/B $(date +%T)"
AB_ARGS="--no-teacher-rate" bash tools/ab_env.sh "KD_PREFETCH_W=0" "KD_PREFETCH_W=1" "KD_PREFETCH_W=0" "KD_PREFETCH_W=1" || exit 1
echo "done2 $(date +%T)"
