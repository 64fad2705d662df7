S="c:1024:16:32:22 c:1024:16:32:6 c:1024:16:16:6 c:1024:32:16:8 c:512:32:32:6 c:512:32:32:0 c:1024:16:16:0"
for pd in 1 2; do echo "== PD $pd"; PG_HR_PD=$pd timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu; done
