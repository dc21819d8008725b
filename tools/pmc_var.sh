# PMC passes on one GEMM shape for each variant in VARS (kd_gemm), one rocprofv3 run per counter set
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
M=${M:-6144}; N=${N:-37888}; K=${K:-3584}; LAY=${LAY:-nt}
for v in ${VARS:-5 16}; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
             "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_MFMA" \
             "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${LAY}_v$v/p$i -o p -- python3 tools/gemm_one.py $M $N $K $v $LAY 5 > gpurun_out/pmc_${LAY}_v${v}_p$i.log 2>&1 || { echo "pmc v$v p$i failed"; tail -5 gpurun_out/pmc_${LAY}_v${v}_p$i.log; exit 1; }
  done
done
echo pmc done
