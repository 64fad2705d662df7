# persistent conv grid (workgroups per CU) sweep at the persistent-tile shapes
cd "$(dirname "$0")/.."
S="c:1024:16:32:6 c:1024:16:32:8 c:1024:16:32:22 c:1024:16:16:6 c:1024:16:16:8 c:1024:32:16:8 c:512:32:32:6 c:512:32:32:0 c:512:32:16:8"
for r in 1 2; do for v in 0 2 3 4 6 8 12; do
  echo "== $v"; if [ $v = 0 ]; then unset PG_HR_PERCU; else export PG_HR_PERCU=$v; fi
  timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu || exit 1
done; done
