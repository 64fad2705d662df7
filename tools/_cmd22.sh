set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); export TMPDIR=/tmp
timeout -k 10 120 python tools/glue_bench.py --iters 1 --check ab/lib_unpoolv.so || exit 1
for v in new=pggan_amd/libpggan_hip.so old=ab/lib_unpoolv.so; do
  name=${v%%=*}; lib=${v#*=}; rm -rf gpurun_out/gb_$name
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/gb_$name" -o run -- python "$ROOT/tools/glue_bench.py" --lib "$ROOT/$lib" ) > gpurun_out/gb_$name.log 2>&1 || { echo "$name failed"; exit 1; }
done
for n in new old; do echo "== $n"; python - <<PY
import csv,collections
d=collections.defaultdict(list)
for r in csv.DictReader(open('gpurun_out/gb_$n/run_kernel_trace.csv')):
    k=r['Kernel_Name']
    if 'unpool' in k: d[(k.split('(')[0][-30:],r['Grid_Size_X'],r['Grid_Size_Y'])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in d.items(): v.sort(); print(k, len(v), 'med', v[len(v)//2])
PY
done
