# A/B of the attention kernels: the in-tree library vs tools/variants/libkdstep_old.so
#   bash tools/ab_attn.sh "student siglip" bwd   (under gpurun)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for shape in $1; do
  for lib in new old; do
    if [ $lib = old ]; then export KDSTEP_LIB=$PWD/tools/variants/libkdstep_old.so; else unset KDSTEP_LIB; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/${shape}_$2_$lib -o run -- python3 tools/attn_one.py $shape 30 $2 > gpurun_out/ab/${shape}_$2_$lib.log 2>&1 || { echo "fail $shape $lib"; exit 1; }
    f=$(ls gpurun_out/ab/${shape}_$2_$lib/*kernel_stats.csv gpurun_out/ab/${shape}_$2_$lib/*/*kernel_stats.csv 2>/dev/null | head -1)
    echo "== $shape $2 $lib"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'attn' in r['Name']: print(f\"{float(r['AverageNs'])/1e3:9.1f} us {int(r['Calls']):4d}  {r['Name'][:90]}\")"
  done
done
