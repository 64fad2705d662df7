"""Checkpoints in the reference's file layout (lib/checkpoint.py:5-34):
{save_root}/{run_id}/ckpt/{G,D}_{step}.pt and {G,D}_latest.pt, holding the schedule
scalars + 'args' + 'model' (reference state_dict keys) + 'optimizer'
(torch.optim.Adam state_dict layout).  Loading uses weights_only=True."""
import os

import torch

from .config import cfg_get


def save_checkpoint(model, optimizer, name, ckpt_dict):
    ckpt_dict["model"] = {k: v.detach().clone() for k, v in model.state_dict().items()}
    ckpt_dict["optimizer"] = optimizer.state_dict()
    args = ckpt_dict["args"]
    dir_path = f'{args["save_root"]}/{args["run_id"]}/ckpt'
    os.makedirs(dir_path, exist_ok=True)
    torch.save(ckpt_dict, f'{dir_path}/{name}_{ckpt_dict["global_step"]}.pt')
    torch.save(ckpt_dict, f"{dir_path}/{name}_latest.pt")


def load_checkpoint(args, name, device="cpu"):
    step = cfg_get(args, "ckpt_step", None)
    step = "latest" if step is None else step
    path = f"{args.save_root}/{args.ckpt_id}/ckpt/{name}_{step}.pt"
    try:
        return torch.load(path, map_location=device, weights_only=True)
    except FileNotFoundError:
        if cfg_get(args, "isMaster", False):
            print(f"Failed to load checkpoint of {name}.")
        return 0
