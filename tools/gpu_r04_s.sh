# round-4 GPU pass S: register-resident KD loss with 3 chunks per lane (3 workgroups/CU) vs 5 (2/CU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== tests $(date +%T)"
KD_LOSS_RR_C=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kd_loss_gpu.py > gpurun_out/s_test3.log 2>&1 || { echo "test rc3 failed"; tail -30 gpurun_out/s_test3.log; exit 1; }
tail -2 gpurun_out/s_test3.log
for rc in 5 3 5 3; do
  KD_LOSS_RR_C=$rc timeout -k 10 200 python -u tools/bench_loss.py 4 loca 2>&1 | grep -v amdgpu.ids | sed "s/^/rc=$rc /" || exit 1
done
echo "done $(date +%T)"
