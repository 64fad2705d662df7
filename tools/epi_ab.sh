# A/B: LDS-staged epilogue (default) vs the direct epilogue (PG_HR_DIAG=8) of the 64-channel DMA tiles
S="c:128:128:128:6 c:128:128:128:8 c:64:256:256:6 c:32:512:512:0 c:256:64:64:6 c:256:64:64:8 c:128:256:128:8 c:256:64:128:22 c:512:32:64:16 c:256:128:64:8 c:64:512:256:8 c:128:128:256:22"
for d in 8 0 8 0; do echo "== diag $d"; PG_HR_DIAG=$d timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu.ids || exit 1; done
