# PMC passes over tools/bench_loss.py (loss kernels only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_TRANS"; do
  i=$((i+1))
  rm -rf gpurun_out/lp/p$i
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/lp/p$i -o p -- python3 tools/bench_loss.py 4 loca > gpurun_out/lp_p$i.log 2>&1 || { echo "pmc p$i failed"; tail -5 gpurun_out/lp_p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/lp/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "kd::" in r["Kernel_Name"]:
            agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:42s} {c:22s} {sum(v)/len(v):.4g}")
PY
