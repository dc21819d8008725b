# PMC passes for one GEMM shape, v3 (variant 5) vs v4 (variant 8); counters in separate passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
M=${1:-6144}; N=${2:-37888}; K=${3:-3584}
for v in 5 8; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_v$v/p$i -o p -- python3 tools/gemm_one.py $M $N $K $v nt 5 > gpurun_out/pmc_v${v}_p$i.log 2>&1 || { echo "pmc v$v p$i failed"; tail -5 gpurun_out/pmc_v${v}_p$i.log; exit 1; }
  done
done
echo pmc done
