# Our GEMM (kd_gemm, v8) vs torch.mm (hipBLASLt) on the two largest step shapes: effective clock
# (GRBM_GUI_ACTIVE / 8 / wall), MFMA busy cycles, wave cycles, SQ busy — one --pmc pass per
# program (SQ 3 + GRBM 1 counters), kernel trace for the wall time.
#   bash tools/pmc_vs_blas.sh  ->  gpurun_out/pmc_blas/*
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_blas
for shape in "6144 37888 3584" "6144 152064 3584"; do
  tag=$(echo $shape | tr ' ' x)
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace \
    --output-format csv -d gpurun_out/pmc_blas/ours_$tag -o p -- python3 tools/gemm_one.py $shape 16 nt 10 \
    > gpurun_out/pmc_blas/ours_$tag.log 2>&1 || { echo "pmc ours $tag failed"; tail -5 gpurun_out/pmc_blas/ours_$tag.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace \
    --output-format csv -d gpurun_out/pmc_blas/blas_$tag -o p -- python3 tools/torch_mm_one.py $shape 10 \
    > gpurun_out/pmc_blas/blas_$tag.log 2>&1 || { echo "pmc blas $tag failed"; tail -5 gpurun_out/pmc_blas/blas_$tag.log; exit 1; }
done
python3 tools/pmc_vs_blas.py gpurun_out/pmc_blas > gpurun_out/pmc_blas/summary.txt && cat gpurun_out/pmc_blas/summary.txt
