# round-4 GPU pass AB: attention backward writing the fused dqkv directly (SigLIP) -- tests and c1 step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_kd_step_gpu.py tests/test_c_host_gpu.py > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
echo "== step A/B $(date +%T)"
AB_ARGS="--no-teacher-rate" bash tools/ab_env.sh "KD_ATTN_DQKV=0" "KD_ATTN_DQKV=1" "KD_ATTN_DQKV=0" "KD_ATTN_DQKV=1" || exit 1
echo "done $(date +%T)"
