# A/B of bench.py under environment settings: AB="VAR=a VAR=b ..." (one bench run each)
set -o pipefail
cd $GRAFT_REPO_ROOT
for kv in $AB; do
  timeout -k 10 300 env $kv python bench.py --no-cpu-baseline --no-timer ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { echo "bench failed ($kv)"; tail -20 gpurun_out/ab.log; exit 1; }
  echo "$kv $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
