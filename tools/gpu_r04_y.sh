# round-4 GPU pass Y: v8 stamps on backward GEMM layouts (MN-major operands) vs the forward layout
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for args in "6144 4608 3584 nt" "6144 4608 3584 nn" "6144 4608 3584 tn" "6144 1024 9728 nn" "9728 1024 6144 tn" "1280 4352 5888 tn"; do
  timeout -k 10 120 python -u tools/stamp_gemm.py $args 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "done $(date +%T)"
