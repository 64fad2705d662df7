"""Training launcher with the reference's entry point (`python train.py <run_id>`,
train.py:69-94) and loop (train.py:11-66), running the MI355X step engine.

Multi-GPU: launch one process per GPU with torch.distributed.run
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        train.py <run_id> [config.yaml]
(the reference uses mp.spawn + a discarded DDP wrapper; here gradients really are
all-reduced over RCCL).
"""
import os
import sys

# One process per GPU with the DP gradient exchange: RCCL's stream and the engine's two
# streams must not share a hardware queue (HIP's default is 4 per process): a collective's
# wait-on-event barrier in a shared queue stalls the compute kernels queued behind it
# (bench.py --dp-exchange at one rank: -16 % of the step with 4 queues, -4 % with 8 or 16,
# profiles/r3_dp_queues.txt; round 6: -2.0 % with 8, -2.2 % with 16, the plain step itself
# -0.75 % at 16, profiles/r6_dp_lines.txt).  Must be set before the HIP runtime starts.
if int(os.environ.get("WORLD_SIZE", "1")) > 1 or "--dp-exchange" in sys.argv:
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from pggan_amd.config import Config  # noqa: E402
from pggan_amd.model import ProgressiveGAN  # noqa: E402


def create_model(rank, args):
    """lib/model_loader.py:4-38 (CreateModel)."""
    args.isMaster = rank == 0
    model = ProgressiveGAN(args, rank)
    model.initialize_models()
    if args.use_mGPU:
        model.set_multi_GPU()
    model.set_optimizers()
    model.set_dataset()
    model.set_data_iterator()
    model.set_loss_collector()
    model.set_validation()
    if args.ckpt_id:
        model.load_checkpoint()
    return model


def train(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    args.use_mGPU = bool(args.use_mGPU) or world > 1
    args.gpu_num = world
    torch.cuda.set_device(local)
    resumed = bool(args.ckpt_id)
    model = create_model(local, args)
    if not resumed:
        model.alpha_index = 0
        model.scale_index = 0
        model.alpha_jump_value = 0
        model.next_scale_jump_step = args.max_step_at_scale[0]
        model.next_alpha_jump_step = args.alpha_jump_start[0]
    step = model.global_step if resumed else 0
    max_step = min(sum(args.max_step_at_scale), args.max_step)
    while step < max_step:
        model.check_jump(step)
        images = model.train_step()
        if rank == 0:
            if step % args.loss_cycle == 0:
                model.loss_collector.print_loss(step)
            if step % args.test_cycle == 0:
                model.save_image(images, step)
            if step % args.ckpt_cycle == 0:
                model.save_checkpoint(step)
        step += 1


if __name__ == "__main__":
    cfg = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "pggan_amd",
                                                              "default_config.yaml")
    args = Config.from_yaml(cfg)
    args.run_id = sys.argv[1] if len(sys.argv) > 1 else args.get("run_id", "run")
    if isinstance(args.get("beta1"), int):
        args.beta1 = float(args.beta1)
    os.makedirs(f"{args.save_root}/{args.run_id}", exist_ok=True)
    train(args)
