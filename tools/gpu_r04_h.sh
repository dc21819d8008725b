# round-4 GPU pass H: RR loss (v1 layout) again + k_row_stats grid A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== loss tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_kd_loss_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_loss.log 2>&1 || { echo "loss tests failed"; tail -40 gpurun_out/t_loss.log; exit 1; }
tail -2 gpurun_out/t_loss.log
echo "== loss A/B $(date +%T)"
for cfg in "KD_LOSS_RR=0 KD_RS_GRID=2048" "KD_LOSS_RR=1 KD_RS_GRID=2048" "KD_LOSS_RR=1" "KD_LOSS_RR=1 KD_RS_GRID=1536" "KD_LOSS_RR=0 KD_RS_GRID=2048" "KD_LOSS_RR=1" ; do env $cfg timeout -k 10 120 python -u tools/bench_loss.py 4 loca 2>&1 | grep kd_loss | sed "s/^/$cfg: /" || exit 1; done
echo "== loss trace $(date +%T)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_loss_h -o run -- python3 tools/bench_loss.py 4 loca > gpurun_out/prof_loss_h.log 2>&1 || { echo "loss trace failed"; tail -5 gpurun_out/prof_loss_h.log; exit 1; }
grep -E "k_loss_grad|k_row_stats" gpurun_out/prof_loss_h/run_kernel_stats.csv | cut -c1-60,200-400 | head
echo "done $(date +%T)"
