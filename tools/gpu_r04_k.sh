# round-4 GPU pass K: six-wave attention forward (variant 36): bit-exactness, A/B vs four waves (32)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== attn tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "six_waves or test_attn_fwd" > gpurun_out/t_attn.log 2>&1 || { echo "attn tests failed"; tail -40 gpurun_out/t_attn.log; exit 1; }
tail -2 gpurun_out/t_attn.log
echo "== attn A/B $(date +%T)"
for v in 32 36 32 36; do KD_ATTN_FWD_V=$v timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids | sed "s/^/V=$v /" || exit 1; done
echo "done $(date +%T)"
