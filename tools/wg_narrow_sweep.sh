# GPU box: narrow weight-gradient variants (PG_WG_VARIANT = "pd,wpe") at 512^2 / 1024^2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S1="w:1024:16:16:0 w:512:32:32:0"
S2="w:512:32:64:0 w:1024:16:32:0"
for v in "2,2" "2,1" "1,2"; do
  echo "== variant '$v'" >> gpurun_out/wgn.txt
  PG_WG_VARIANT=$v timeout -k 10 120 python tools/kbench.py $S1 >> gpurun_out/wgn.txt 2>&1
done
for v in "4,1" "2,1" "2,2"; do
  echo "== variant '$v' (MO 2/4)" >> gpurun_out/wgn.txt
  PG_WG_VARIANT=$v timeout -k 10 120 python tools/kbench.py $S2 >> gpurun_out/wgn.txt 2>&1
done
echo sweep done
