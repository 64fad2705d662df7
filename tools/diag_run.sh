S="c:128:128:128:6 c:64:256:256:6 c:32:512:512:0 c:256:64:64:6 c:128:256:128:8"
for d in 0 1 2 3 4 7; do echo "== diag $d"; PG_HR_DIAG=$d timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu.ids || exit 1; done
