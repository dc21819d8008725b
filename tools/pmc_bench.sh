# rocprofv3 --pmc passes over a short serialized bench (tools/gpu_round.sh steps pmc / pmcstep).
#   OUT=gpurun_out/r05 bash tools/pmc_bench.sh          HBM traffic: FETCH_SIZE and WRITE_SIZE in separate
#                                                        passes (MI355X_MICROARCH.md: FETCH_SIZE takes 3 TCC
#                                                        slots, WRITE_SIZE 2) -> $OUT/pmc_traffic.json
#   OUT=gpurun_out/r05 bash tools/pmc_bench.sh mfma     + a pass of GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES,
#                                                        SQ_BUSY_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES (1 GRBM + 3 SQ),
#                                                        folded per kernel family by tools/pmc_step.py
#                                                        -> $OUT/pmc_step.json
# Counters only (no trace domains beside them); every pass has its own hard time limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out}
mkdir -p $OUT/pmc_bench
BENCH="bench.py --steps 2 --warmup 1 --serial --no-teacher-rate --no-cpu-baseline --no-timer --no-delta"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_bench/p$i -o p -- python3 $BENCH > $OUT/pmc_bench_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_bench_p$i.log; exit 1; }
done
python3 tools/pmc_traffic.py $OUT/pmc_bench > $OUT/pmc_traffic.json && head -c 600 $OUT/pmc_traffic.json
if [ "$1" = mfma ]; then
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc_bench/p3 -o p -- python3 $BENCH > $OUT/pmc_bench_p3.log 2>&1 || { echo "pmc pass 3 failed"; tail -5 $OUT/pmc_bench_p3.log; exit 1; }
  # the wall times come from the plain kernel trace of the same serialized bench (gpu_round.sh step prof)
  TRACE=$(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$TRACE" ] || { echo "pmcstep needs the prof step's kernel trace first (STEPS=\"prof pmcstep\")"; exit 1; }
  python3 tools/pmc_step.py $OUT/pmc_bench $TRACE > $OUT/pmc_step.json && head -c 2000 $OUT/pmc_step.json
fi
