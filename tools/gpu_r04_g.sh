# round-4 GPU pass G: pipelined register-resident KD loss (tests, A/B, trace, FETCH) + v12 odd-barrier A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== loss tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_kd_loss_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_loss.log 2>&1 || { echo "loss tests failed"; tail -40 gpurun_out/t_loss.log; exit 1; }
tail -2 gpurun_out/t_loss.log
echo "== loss A/B $(date +%T)"
for rr in 0 1 0 1; do KD_LOSS_RR=$rr timeout -k 10 120 python -u tools/bench_loss.py 4 loca 2>&1 | grep kd_loss | sed "s/^/RR=$rr /" || exit 1; done
echo "== loss trace $(date +%T)"
KD_LOSS_RR=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_loss_rr1b -o run -- python3 tools/bench_loss.py 4 loca > gpurun_out/prof_loss_rr1b.log 2>&1 || { echo "loss trace failed"; tail -5 gpurun_out/prof_loss_rr1b.log; exit 1; }
KD_LOSS_RR=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_loss_rr1b -o p -- python3 tools/bench_loss.py 4 loca > gpurun_out/pmc_loss_rr1b.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_loss_rr1b.log; exit 1; }
echo "== v12 tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gemm_v12_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_v12.log 2>&1 || { echo "v12 tests failed"; tail -40 gpurun_out/t_v12.log; exit 1; }
tail -2 gpurun_out/t_v12.log
echo "== ab $(date +%T)"
timeout -k 10 400 python -u tools/ab_v11.py --rounds 4 --variants 24,26,27 > gpurun_out/ab_v12nb.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_v12nb.log; exit 1; }
grep -v "^{" gpurun_out/ab_v12nb.log | cut -c1-250
echo "done $(date +%T)"
