# SQ counters of the attention backward kernels (both arms of tools/ab_attn_bwd32.py, A/B library).
#   OUT=gpurun_out/bwd32 bash tools/pmc_attn_bwd.sh
# Keeps only the counters rocprofv3 lists on this box; one pass per set of <= 8 SQ counters, each
# under its own hard time limit; counters only (no trace domains beside them).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/bwd32}
mkdir -p $OUT/pmc
timeout -s KILL 60 rocprofv3 -L > $OUT/pmc/avail.txt 2>&1 || { echo "counter list failed"; tail -5 $OUT/pmc/avail.txt; exit 1; }
have() { for c in "$@"; do grep -qw "$c" $OUT/pmc/avail.txt && printf "%s " "$c"; done; }
S1=$(have SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE)
S2=$(have SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM)
echo "set1: $S1"; echo "set2: $S2"
i=0
for set in "$S1" "$S2"; do
  i=$((i+1))
  [ -n "$set" ] || continue
  KDSTEP_LIB=tools/ab/libkdstep_ab.so timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc/p$i -o p \
      -- python3 tools/ab_attn_bwd32.py > $OUT/pmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc/p$i.log; exit 1; }
done
python3 - "$OUT/pmc" <<'EOF'
import csv, glob, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_attn_bwd" not in k:
            continue
        name = k.split("(")[0].replace("void kd::(anonymous namespace)::", "")
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(name, r["Counter_Name"])] += 1
for name, d in sorted(acc.items()):
    calls = max(n[(name, c)] for c in d)
    print(name, {c: round(v / calls) for c, v in sorted(d.items())})
EOF
