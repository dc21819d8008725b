# round-4 GPU pass X: AdamW on fewer CUs (KD_ADAMW_GRID) -- single calls, then the concurrent c1 step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k adamw tests/test_layers_gpu.py tests/test_kd_step_gpu.py > gpurun_out/x_tests.log 2>&1 || { tail -30 gpurun_out/x_tests.log; exit 1; }
tail -1 gpurun_out/x_tests.log
for gr in 0 1024 256 128 64; do
  KD_ADAMW_GRID=$gr timeout -k 10 120 python -u tools/bench_adamw.py 2>&1 | grep -v amdgpu.ids | head -1 | sed "s/^/grid=$gr /" || exit 1
done
echo "== step A/B $(date +%T)"
AB_ARGS="--no-teacher-rate" bash tools/ab_env.sh "KD_ADAMW_GRID=0" "KD_ADAMW_GRID=256" "KD_ADAMW_GRID=128" "KD_ADAMW_GRID=0" "KD_ADAMW_GRID=256" "KD_ADAMW_GRID=128" || exit 1
echo "done $(date +%T)"
