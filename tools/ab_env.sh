# A/B of environment settings on the c1 bench (one line per variant):
#   bash tools/ab_env.sh "" "KD_GEMM_SPLIT_K=1 KD_WGRAD_SPLIT_K=1" ...
# Each variant runs `env <settings> python bench.py` with its own time limit; the first
# failure ends the script.
set -o pipefail
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i + 1))
  env $v timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-delta --no-timer $AB_ARGS > gpurun_out/ab_$i.log 2>&1 || { echo "variant $i failed"; tail -5 gpurun_out/ab_$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1]); print('[$v]', d['value'], d['ms_per_step'])"
done
