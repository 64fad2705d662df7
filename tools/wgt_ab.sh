cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
AB_VAR=PG_WG_TARGET_NARROW AB_A=1024 AB_B=512 bash tools/env_ab2.sh 2 || exit 1

