# round-4 GPU pass V: packed SwiGLU epilogue vs the previous one on one box (single calls, c1 step)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== single calls $(date +%T)"
timeout -k 10 300 python -u tools/ab_glu_epi.py --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
echo "== step A/B $(date +%T)"
AB_ARGS="--no-teacher-rate" bash tools/ab_env.sh "KD_GLU_EPI_V0=1" "KD_GLU_EPI_V0=0" "KD_GLU_EPI_V0=1" "KD_GLU_EPI_V0=0" || exit 1
echo "done $(date +%T)"
