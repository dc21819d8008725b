# SQ counters of the attention kernels (two --pmc passes, one run each):
#   bash tools/pmc_attn.sh student bwd     (under gpurun) -> gpurun_out/pmc_attn_<shape>_<mode>.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/pmcattn_$1_$2
mkdir -p $out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/p1 -o run -- python3 tools/attn_one.py $1 10 $2 > $out/p1.log 2>&1 || { echo "p1 failed"; tail -5 $out/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $out/p2 -o run -- python3 tools/attn_one.py $1 10 $2 > $out/p2.log 2>&1 || { echo "p2 failed"; tail -5 $out/p2.log; exit 1; }
python3 - $out > gpurun_out/pmc_attn_$1_$2.txt <<'PY'
import collections, csv, glob, sys
root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
dur = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("kd::(anonymous namespace)::", "").split("(")[0]
        if "attn" not in n:
            continue
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[n][r["Counter_Name"]] += 1
        if r["Counter_Name"] in ("SQ_WAVES", "GRBM_GUI_ACTIVE"):
            dur[n].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for n, d in agg.items():
    print(n, f"avg dur {sum(dur[n]) / max(1, len(dur[n])) / 1e3:.1f} us")
    for k in sorted(d):
        print(f"   {k:28s} {d[k] / max(1, cnt[n][k]):16.0f}")
PY
cat gpurun_out/pmc_attn_$1_$2.txt
