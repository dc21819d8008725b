# generate() parity tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_generate.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_gen.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pt_gen.log; exit 1; }
tail -3 gpurun_out/pt_gen.log
echo done
