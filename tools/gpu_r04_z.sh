# round-4 GPU pass Z: k_attn_fwd64 (two query blocks per wave) -- bit-exactness and timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "two_blocks or six_waves" tests/test_attention_gpu.py > gpurun_out/z_tests.log 2>&1 || { tail -30 gpurun_out/z_tests.log; exit 1; }
tail -1 gpurun_out/z_tests.log
timeout -k 10 200 python -u tools/ab_attn_fwd.py "0 64" 2>&1 | grep -v amdgpu.ids || exit 1
echo "done $(date +%T)"
