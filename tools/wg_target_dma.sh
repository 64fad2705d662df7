cd "${GRAFT_REPO_ROOT}"
S="w:512:32:32:0 w:512:64:32:1 w:1024:16:32:0 w:1024:16:16:0 w:1024:32:16:1"
for v in "PG_WG_DMA=2" "PG_WG_DMA=3" "PG_WG_DMA=3 PG_WG_TARGET_NARROW=256" "PG_WG_DMA=2 PG_WG_TARGET_NARROW=256" "PG_WG_DMA=2 PG_WG_TARGET_NARROW=1024"; do
  echo "== $v"
  env $v timeout -k 10 120 python tools/kbench.py --iters 20 $S 2>&1 | grep -v amdgpu || exit 1
done
