# GPU box: wide conv_hr tile / staging variants on the 64^2-256^2 shapes (kbench)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S="c:128:128:128:6 c:64:256:256:6 c:256:64:64:6 c:256:128:64:8 c:128:256:128:8 c:64:512:256:8"
for v in "PG_HR_TILE=-1" "PG_HR_TILE=3" "PG_HR_TILE=6" "PG_HR_DMA=0" "PG_HR_TILE=6 PG_HR_DMA=0"; do
  echo "== $v" >> gpurun_out/hrw.txt
  env $v timeout -k 10 120 python tools/kbench.py $S >> gpurun_out/hrw.txt 2>&1 || exit 1
done
PMC_SPECS="c:128:128:128:6" bash tools/pmc_hr.sh
