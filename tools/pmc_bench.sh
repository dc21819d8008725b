# HBM traffic of the bench step's kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3
# --pmc passes (MI355X_MICROARCH.md: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2), folded per
# kernel by tools/pmc_traffic.py (gfx950 FETCH_SIZE x2 correction) into gpurun_out/pmc_traffic.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_bench/p$i -o p -- python3 bench.py --steps 2 --warmup 1 --serial --no-teacher-rate --no-cpu-baseline --no-timer --no-delta > gpurun_out/pmc_bench_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_bench_p$i.log; exit 1; }
done
python3 tools/pmc_traffic.py gpurun_out/pmc_bench > gpurun_out/pmc_traffic.json && head -c 1500 gpurun_out/pmc_traffic.json
