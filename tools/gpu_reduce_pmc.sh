# PMC + kernel trace of one split-K GEMM (auto plan) to study the split-K reduce kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
M=${M:-896}; N=${N:-4864}; K=${K:-6144}; LAY=${LAY:-tn}
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/red/kt -o k -- python3 tools/gemm_one.py $M $N $K 0 $LAY 10 > gpurun_out/red_kt.log 2>&1 || { echo kt failed; tail -5 gpurun_out/red_kt.log; exit 1; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/red/p$i -o p -- python3 tools/gemm_one.py $M $N $K 0 $LAY 5 > gpurun_out/red_p$i.log 2>&1 || { echo "pmc p$i failed"; tail -5 gpurun_out/red_p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/red/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:60s} {c:22s} {sum(v)/len(v):.4g}")
for f in glob.glob("gpurun_out/red/kt/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
