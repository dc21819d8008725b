# round-4 GPU pass P: fp8 teacher vs the reference at the real widths
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== fp8 tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "real_widths_vs_reference" > gpurun_out/t_fp8_ref.log 2>&1; rc=$?
grep -E "fp8 |PASS|FAIL|passed|failed|Error" gpurun_out/t_fp8_ref.log | cut -c1-300 | tail -20
exit $rc
