# conv_hr ring depth and wgrad (prefetch depth, waves/SIMD) sweeps at the 1024^2-256^2 shapes
S="c:1024:16:32:22 c:1024:16:32:8 c:1024:16:16:6 c:1024:16:16:8 c:1024:32:16:8 c:512:32:32:6 c:512:32:64:22 c:512:64:32:8"
for pd in 1 2 3; do echo "== PD $pd"; PG_HR_PD=$pd timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu || exit 1; done
W="w:1024:16:32:0 w:1024:16:16:0 w:1024:32:16:1 w:512:32:64:0 w:512:32:32:0 w:256:64:128:0 w:256:64:64:0"
for v in 2,2 4,1 2,1 1,2; do echo "== WG $v"; PG_WG_VARIANT=$v timeout -k 10 120 python tools/kbench.py $W 2>&1 | grep -v amdgpu || exit 1; done
