# A/B: persistent 64-wide conv_hr tiles (14: cin 32, 15: cin 64) vs the default tile
A="c:512:32:64:22 c:512:32:64:16"
Bs="c:256:64:64:6 c:256:64:64:8 c:256:64:64:0"
echo "== default"; timeout -k 10 120 python tools/kbench.py $A $Bs 2>&1 | grep -v amdgpu.ids || exit 1
for pd in 1 2; do
echo "== tile14 pd $pd"; PG_HR_PD=$pd PG_HR_TILE=14 timeout -k 10 120 python tools/kbench.py $A 2>&1 | grep -v amdgpu.ids || exit 1
echo "== tile15 pd $pd"; PG_HR_PD=$pd PG_HR_TILE=15 timeout -k 10 120 python tools/kbench.py $Bs 2>&1 | grep -v amdgpu.ids || exit 1
done
