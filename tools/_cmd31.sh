set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
bash tools/ab.sh -r 4 "base:" "hipri:PG_MAIN_HIPRI=1"; grep round gpurun_out/ab.log
