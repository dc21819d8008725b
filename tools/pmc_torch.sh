set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_torch/p$i -o p -- python3 tools/torch_mm_one.py 6144 37888 3584 5 > gpurun_out/pmc_torch_p$i.log 2>&1 || { echo "pmc p$i failed"; tail -5 gpurun_out/pmc_torch_p$i.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_torch/kt -o k -- python3 tools/torch_mm_one.py 6144 37888 3584 5 > gpurun_out/pmc_torch_kt.log 2>&1 || { echo kt failed; exit 1; }
echo done
