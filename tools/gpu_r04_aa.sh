# round-4 GPU pass AA: norm forward with hoisted loads -- bit-exactness, single calls, c1 step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "norm" tests/test_layers_gpu.py > gpurun_out/aa_tests.log 2>&1 || { tail -30 gpurun_out/aa_tests.log; exit 1; }
tail -1 gpurun_out/aa_tests.log
timeout -k 10 200 python -u tools/ab_norm_fwd.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== step A/B $(date +%T)"
AB_ARGS="--no-teacher-rate" bash tools/ab_env.sh "KD_NORM_FWD_V=1" "KD_NORM_FWD_V=2" "KD_NORM_FWD_V=1" "KD_NORM_FWD_V=2" || exit 1
echo "done $(date +%T)"
