cd $GRAFT_REPO_ROOT
S="c:32:512:512:8 c:32:512:512:6 c:16:512:512:6 c:16:512:512:8 c:8:512:512:6 c:4:512:512:6 c:64:256:512:22 c:64:512:256:8"
for r in 1 2; do
for v in "128,256" "512,512" "512,768" "512,1024" "128,512" "128,1024"; do
  echo "== $v"; PG_CONV_SPLIT=$v timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu || exit 1
done; done
