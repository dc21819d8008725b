# Round-end style GPU pass (run under gpurun):
#   STEPS="tests parity bench prof pmc" ROUND=r02 bash tools/gpu_round.sh
# smoke  : __graft_entry__.smoke()
# tests  : pytest -m gpu (every parity test); gemm: only the GEMM / fp8 GEMM tests
# c2, c4 : bench.py --config c2 / c4 (the other single-GPU BASELINE configs) -> gpurun_out/bench_c*.log
# parity : tools/parity_report.py -> gpurun_out/parity.json (per-term deltas vs the reference)
# bench  : python bench.py (the driver's default line) -> gpurun_out/bench.log
# prof   : rocprofv3 --kernel-trace --stats of a serialized bench (its roofline-kernel average
#          is what bench.py's HIP-event pass measures)
# step   : kernel trace of the concurrent (default) bench -> gpurun_out/step_breakdown.txt
# blas   : PMC clock / MFMA-busy of kd_gemm vs hipBLASLt on the two big shapes (tools/pmc_vs_blas.sh)
# pmc    : HBM traffic per kernel (tools/pmc_bench.sh, two --pmc passes)
# Every step has its own time limit; the first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
STEPS=${STEPS:-"tests parity bench prof"}
BENCH_ARGS=${BENCH_ARGS:-""}
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    smoke)  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
            tail -1 gpurun_out/smoke.log ;;
    tests)  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
            tail -2 gpurun_out/pytest_gpu.log ;;
    parity) timeout -k 10 600 python -u tools/parity_report.py --out gpurun_out/parity.json $PARITY_KINDS > gpurun_out/parity.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/parity.log; exit 1; } ;;
    bench)  timeout -k 10 900 python -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
            tail -1 gpurun_out/bench.log ;;
    c2|c4)  timeout -k 10 600 python -u bench.py --config $s --no-cpu-baseline > gpurun_out/bench_$s.log 2>&1 || { echo "bench $s failed"; tail -30 gpurun_out/bench_$s.log; exit 1; }
            tail -1 gpurun_out/bench_$s.log | cut -c1-240 ;;
    gemm)   timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/pytest_gemm.log; exit 1; }
            tail -1 gpurun_out/pytest_gemm.log ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --serial --no-teacher-rate --no-cpu-baseline --no-delta $BENCH_ARGS > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; } ;;
    step)   timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/profstep -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-delta --no-timer --no-teacher-rate $BENCH_ARGS > gpurun_out/profstep.log 2>&1 || { echo "profstep failed"; tail -20 gpurun_out/profstep.log; exit 1; }
            python3 tools/step_breakdown.py $(ls gpurun_out/profstep/*/run_results.db gpurun_out/profstep/run_results.db 2>/dev/null | head -1) 40 > gpurun_out/step_breakdown.txt 2>&1; head -45 gpurun_out/step_breakdown.txt ;;
    blas)   bash tools/pmc_vs_blas.sh > gpurun_out/pmc_blas.log 2>&1 || { echo "pmc_vs_blas failed"; tail -10 gpurun_out/pmc_blas.log; exit 1; }
            cat gpurun_out/pmc_blas/summary.txt ;;
    pmc)    bash tools/pmc_bench.sh > gpurun_out/pmc_bench.log 2>&1 || { echo "pmc failed"; tail -10 gpurun_out/pmc_bench.log; exit 1; } ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "done $(date +%T)"
