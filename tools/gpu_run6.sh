set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/fp8_depth_study.py --depths 8,28 --families all,lm,lm_body,lm_mlp --out gpurun_out/fp8_depth.json > gpurun_out/fp8_depth.log 2>&1 || { echo "fp8 study failed"; tail -20 gpurun_out/fp8_depth.log; exit 1; }
cat gpurun_out/fp8_depth.log | grep depth
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not test_training_step_matches_reference" > gpurun_out/pytest_rest.log 2>&1; echo "rc=$?"; tail -5 gpurun_out/pytest_rest.log
