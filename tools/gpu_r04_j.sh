# round-4 GPU pass J: c3 and c4 bench lines, attention forward stamps (teacher causal, SigLIP)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in c3 c4; do
  echo "== bench $c $(date +%T)"
  timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -30 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | cut -c1-300
done
echo "== stamps $(date +%T)"
KD_ATTN_FWD_V=34 timeout -k 10 120 python -u tools/stamp_attn.py 4 28 4 1536 128 128 1 > gpurun_out/stamp_teacher.log 2>&1 || { echo "stamp failed"; tail -10 gpurun_out/stamp_teacher.log; exit 1; }
KD_ATTN_FWD_V=34 timeout -k 10 120 python -u tools/stamp_attn.py 8 16 16 729 72 96 0 > gpurun_out/stamp_siglip.log 2>&1 || { echo "stamp failed"; tail -10 gpurun_out/stamp_siglip.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamp_teacher.log gpurun_out/stamp_siglip.log
echo "done $(date +%T)"
