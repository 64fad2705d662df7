cd "$(dirname "$0")/.."
S="w:512:32:64:0 w:256:64:128:0 w:256:64:64:0 w:128:128:256:0 w:128:128:128:0 w:64:256:512:0 w:64:256:256:0 w:32:512:512:0 w:16:512:512:0 w:8:512:512:0"
for r in 1 2; do for v in 1 2; do
  echo "== $v"; PG_WG_WNC=$v timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu || exit 1
  PG_WG_WNC=$v PG_WG_BP=128 timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu | sed 's/^/bp128:/' || exit 1
done; done
