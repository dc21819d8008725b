# round-4 GPU pass O: c1 A/B of the GEMM plan (round-3 warm constants vs round-4 cold constants, hybrid on/off)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== plan A/B $(date +%T)"
AB_ARGS="--no-teacher-rate" bash tools/ab_env.sh "KD_PLAN_SET=3" "KD_PLAN_SET=4" "KD_PLAN_SET=4 KD_GEMM_HYBRID=0" "KD_PLAN_SET=3 KD_GEMM_HYBRID=0" "KD_PLAN_SET=3" "KD_PLAN_SET=4" "KD_PLAN_SET=4 KD_GEMM_HYBRID=0" "KD_PLAN_SET=3 KD_GEMM_HYBRID=0" || exit 1
echo "done $(date +%T)"
