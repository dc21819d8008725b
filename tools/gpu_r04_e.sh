# round-4 GPU pass E: smoke, the register-resident KD loss (tests, A/B, kernel trace, FETCH_SIZE),
# the default bench line and its serialized rocprofv3 kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== loss tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_kd_loss_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_loss.log 2>&1 || { echo "loss tests failed"; tail -40 gpurun_out/t_loss.log; exit 1; }
tail -2 gpurun_out/t_loss.log
echo "== loss A/B $(date +%T)"
for rr in 0 1 0 1; do KD_LOSS_RR=$rr timeout -k 10 120 python -u tools/bench_loss.py 4 loca 2>&1 | grep kd_loss | sed "s/^/RR=$rr /" || exit 1; done
echo "== loss trace $(date +%T)"
for rr in 0 1; do KD_LOSS_RR=$rr timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_loss_rr$rr -o run -- python3 tools/bench_loss.py 4 loca > gpurun_out/prof_loss_rr$rr.log 2>&1 || { echo "loss trace failed"; tail -5 gpurun_out/prof_loss_rr$rr.log; exit 1; }; done
for rr in 0 1; do f=$(ls gpurun_out/prof_loss_rr$rr/*/run_kernel_stats.csv gpurun_out/prof_loss_rr$rr/run_kernel_stats.csv 2>/dev/null | head -1); echo "RR=$rr $f"; cut -d, -f1-4 "$f" | head -8; done
echo "== loss FETCH $(date +%T)"
KD_LOSS_RR=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_loss_rr1 -o p -- python3 tools/bench_loss.py 4 loca > gpurun_out/pmc_loss_rr1.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_loss_rr1.log; exit 1; }
KD_LOSS_RR=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_loss_rr1w -o p -- python3 tools/bench_loss.py 4 loca > gpurun_out/pmc_loss_rr1w.log 2>&1 || { echo "pmc w failed"; tail -5 gpurun_out/pmc_loss_rr1w.log; exit 1; }
echo "== bench $(date +%T)"
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-600
echo "== prof $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --serial --no-teacher-rate --no-cpu-baseline --no-delta > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
tail -1 gpurun_out/prof.log | cut -c1-300
echo "done $(date +%T)"
