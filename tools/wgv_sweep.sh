cd "$(dirname "$0")/.."
S="w:512:32:64:0 w:256:64:128:0 w:256:64:64:0 w:128:128:256:0 w:128:128:128:0 w:64:256:512:0 w:64:256:256:0 w:32:512:512:0"
for r in 1 2; do for v in 4,1 2,1 2,2; do for t in 256 512; do
  echo "== $v/$t"; PG_WG_VARIANT=$v PG_WG_TARGET=$t timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu || exit 1
done; done; done
