set -o pipefail
cd $GRAFT_REPO_ROOT
S="c:256:64:64:0 c:256:64:64:6 c:256:128:64:8 c:128:128:128:0 c:128:128:128:6 c:128:256:128:8 c:64:256:256:0 c:64:512:256:8 c:64:256:256:6"
for B in 4 8; do
  for v in base multi base multi; do
    if [ $v = multi ]; then L="--lib ab/lib_multi.so"; else L=""; fi
    timeout -k 10 200 python tools/kbench.py --B $B --iters 30 $L $S 2>&1 | grep -v amdgpu.ids | sed "s/^/B$B $v /"
  done
done
