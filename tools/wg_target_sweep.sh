# GPU box: pixel-split target of the narrow weight gradients (PG_WG_TARGET)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S="w:512:32:32:0 w:1024:16:16:0 w:1024:16:32:0 w:512:32:64:0 w:256:64:64:0 w:32:512:512:0 w:16:512:512:0 w:8:512:512:0"
echo "== target default" >> gpurun_out/wgt.txt
timeout -k 10 120 python tools/kbench.py $S >> gpurun_out/wgt.txt 2>&1
for t in 256 512 2048; do
  echo "== target $t" >> gpurun_out/wgt.txt
  PG_WG_TARGET=$t timeout -k 10 120 python tools/kbench.py $S >> gpurun_out/wgt.txt 2>&1
done
echo sweep done
