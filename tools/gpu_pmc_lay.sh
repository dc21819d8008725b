set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread -k norm > gpurun_out/pt_norm.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_norm.log; exit 1; }
tail -2 gpurun_out/pt_norm.log
M=5832 N=4304 K=1152 VARS="5" LAY=nt bash tools/pmc_var.sh && M=5832 N=4304 K=1152 VARS="5" LAY=nn bash tools/pmc_var.sh && M=5832 N=4304 K=1152 VARS="5" LAY=tn bash tools/pmc_var.sh
python tools/pmc_summary.py gpurun_out/pmc_nt_v5 gpurun_out/pmc_nn_v5 gpurun_out/pmc_tn_v5
