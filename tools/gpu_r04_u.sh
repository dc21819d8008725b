# round-4 GPU pass U: the packed SwiGLU epilogue -- bit-exactness, stamps, the c1 step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "swiglu or glu" \
  tests/test_gemm_gpu.py tests/test_gemm_v11_gpu.py tests/test_gemm_v12_gpu.py tests/test_layers_gpu.py \
  tests/test_bench_shapes_gpu.py tests/test_fp8_gpu.py tests/test_gemm_pretiled_gpu.py > gpurun_out/u_tests.log 2>&1 || { tail -40 gpurun_out/u_tests.log; exit 1; }
tail -2 gpurun_out/u_tests.log
echo "== stamps $(date +%T)"
timeout -k 10 200 python -u tools/stamp_glu.py 6144 37888 3584 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -u tools/stamp_glu.py 6144 9728 896 --aux 2>&1 | grep -v amdgpu.ids || exit 1
echo "== bench c1 $(date +%T)"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/u_bench.json 2> gpurun_out/u_bench.err || { tail -20 gpurun_out/u_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/u_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']); print(d.get('gemm_breakdown',{}).get('gemm_kk_swiglu'))"
echo "done $(date +%T)"
