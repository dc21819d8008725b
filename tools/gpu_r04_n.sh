# round-4 GPU pass N: the plan's candidates timed in the step's cache state (tools/tune_gemm_cold.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== cold tune $(date +%T)"
timeout -k 10 900 python -u tools/tune_gemm_cold.py tools/step_shapes_c1.json 60 --iters 6 > gpurun_out/gemm_tune_cold.jsonl 2> gpurun_out/gemm_tune_cold.err || { echo "tune failed"; tail -20 gpurun_out/gemm_tune_cold.err; exit 1; }
wc -l gpurun_out/gemm_tune_cold.jsonl
echo "done $(date +%T)"
