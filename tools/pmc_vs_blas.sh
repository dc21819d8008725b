# Our GEMM (kd_gemm, v8) vs torch.mm (hipBLASLt) on the two largest step shapes: effective clock
# (GRBM_GUI_ACTIVE / 8 / wall), MFMA busy cycles, wave cycles, SQ busy -- one --pmc pass per
# program (SQ 3 + GRBM 1 counters) -- and FETCH_SIZE / WRITE_SIZE in passes of their own
# (L2 -> fabric bytes per launch: how much each kernel re-reads from beyond L2).
#   OUT=gpurun_out/r05 bash tools/pmc_vs_blas.sh  ->  $OUT/pmc_blas/*
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out}
mkdir -p $OUT/pmc_blas
for shape in "6144 37888 3584" "6144 152064 3584"; do
  tag=$(echo $shape | tr ' ' x)
  for prog in ours blas; do
    if [ $prog = ours ]; then cmd="tools/gemm_one.py $shape 16 nt 10"; else cmd="tools/torch_mm_one.py $shape 10"; fi
    timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
      --output-format csv -d $OUT/pmc_blas/${prog}_$tag -o p -- python3 $cmd \
      > $OUT/pmc_blas/${prog}_$tag.log 2>&1 || { echo "pmc $prog $tag failed"; tail -5 $OUT/pmc_blas/${prog}_$tag.log; exit 1; }
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_blas/${prog}_$tag/$c -o p -- python3 $cmd \
        > $OUT/pmc_blas/${prog}_${tag}_$c.log 2>&1 || { echo "pmc $prog $tag $c failed"; tail -5 $OUT/pmc_blas/${prog}_${tag}_$c.log; exit 1; }
    done
  done
done
python3 tools/pmc_vs_blas.py $OUT/pmc_blas > $OUT/pmc_blas/summary.txt && cat $OUT/pmc_blas/summary.txt
