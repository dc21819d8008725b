# round-4 GPU pass W: gate|up GEMM placement / per-CU gaps / in-kernel clock (stamp build 28)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/stamp_glu.py 6144 37888 3584 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -u tools/stamp_glu.py 6144 9728 896 --aux 2>&1 | grep -v amdgpu.ids || exit 1
echo "done $(date +%T)"
