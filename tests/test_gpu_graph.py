"""The two replayed forms of the training step at world 1 -- the hipGraph capture
(ProgressiveGAN.use_graph) and the library's C++ launch recorder (use_replay, the default) --
against the same model stepped eagerly, after every step, including across a change of alpha
(a new capture / recording), an external parameter edit (load_state_dict: repack + re-record)
and an optimizer state load: BITWISE equal latents, losses, gradients, parameters and Adam
moments.  Every reduction in the library is deterministic (fixed-order combines, no float
atomics), so the same kernels on the same inputs give the same bits however they are issued;
a replay of the wrong step (stale latents, a wrong bias correction) differs everywhere."""
import pytest
import torch

from gen_inputs import TINY_DEPTHS
from test_model_api import make_args

pytestmark = pytest.mark.gpu


def build(args, graph, s):
    from pggan_amd.model import ProgressiveGAN
    ProgressiveGAN.ops_factory = None
    torch.manual_seed(7)
    m = ProgressiveGAN(args, 0)
    m.use_graph = graph         # (opt-in in the product: ProgressiveGAN.use_graph)
    m.use_replay = False        # (the product default; build_replay turns it back on)
    m.initialize_models()
    for i in range(1, s + 1):
        m.G.add_block(args.depths[i])
        m.D.add_block(args.depths[i])
    m.scale_index = s
    m.set_optimizers()
    m.set_dataset()
    m.set_data_iterator()
    m.set_loss_collector()
    return m


def state(m):
    out = {"loss": m._engines[next(iter(m._engines))].loss.clone(), "z": m._z.clone()}
    for n, fp in (("G", m.fpG), ("D", m.fpD)):
        out[n + "p"], out[n + "g"] = fp.flat.clone(), fp.grad.clone()
        out[n + "m"], out[n + "v"] = fp.m.clone(), fp.v.clone()
    return out


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_graph_replay_matches_eager(tmp_path, dtype):
    args = make_args(tmp_path, depths=list(TINY_DEPTHS), compute_dtype=dtype)
    s = 3
    eager, graph = build(args, False, s), build(args, True, s)
    for m in (eager, graph):
        m.G.alpha = m.D.alpha = 0.5
    for step in range(9):
        if step == 4:           # alpha ramp: the graph is recaptured for the new scalars
            for m in (eager, graph):
                m.G.alpha = m.D.alpha = 0.75
        if step == 5:           # external edit: version counters bump -> repack, eager step
            sd = {k: v.clone() * 1.01 for k, v in eager.G.state_dict().items()}
            for m in (eager, graph):
                m.G.load_state_dict(sd)
        if step == 7:           # optimizer state alone: the host Adam count changes, no
            # parameter version does -- the replay must not run with the device's old count
            for m in (eager, graph):
                sd = m.opt_D.state_dict()
                for st in sd["state"].values():
                    st["step"] = torch.tensor(float(m.fpD.step - 2))
                m.opt_D.load_state_dict(sd)
        eager.train_step()
        graph.train_step()
        torch.cuda.synchronize()
        a, b = state(eager), state(graph)
        assert torch.equal(a["z"], b["z"]), step
        assert eager.fpG.step == graph.fpG.step == step + 1
        assert int(graph.fpD.step_dev.item()) == graph.fpD.step
        if step in (2, 3, 8):   # steady state: a captured graph replayed
            assert "graph" in graph._gstate, step
        for k in a:
            assert torch.equal(a[k], b[k]), (step, k, float((a[k].double() - b[k].double()).abs().max()))


def build_replay(args, s):
    m = build(args, False, s)
    m.use_replay = True
    return m


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_cpp_replay_matches_eager_bitwise(tmp_path, dtype):
    """The step recorded by the library's launch recorder and re-issued from C++ (use_replay,
    pg_record_* / pg_replay) against the same model stepped eagerly: BITWISE equal after every
    step -- latents, losses, gradients, parameters, Adam moments -- across an alpha change (a
    new recording), an external parameter edit (repack, eager step, re-record) and an optimizer
    state load (the host step count moves alone).  Same kernels on the same streams, and every
    reduction deterministic, so nothing may differ at all."""
    args = make_args(tmp_path, depths=list(TINY_DEPTHS), compute_dtype=dtype)
    s = 3
    eager, rep = build(args, False, s), build_replay(args, s)
    for m in (eager, rep):
        m.G.alpha = m.D.alpha = 0.5
    replayed = 0
    # step 0 packs the weights (eager), step 1 is the key's first step (eager), step 2 records
    # while it runs, 3-5 replay; alpha changes at 6 (eager, 7 records), the parameter edit at 8
    # and the optimizer load at 10 run eagerly, 11 records again
    for step in range(12):
        if step == 6:
            for m in (eager, rep):
                m.G.alpha = m.D.alpha = 0.75
        if step == 8:
            sd = {k: v.clone() * 1.01 for k, v in eager.G.state_dict().items()}
            for m in (eager, rep):
                m.G.load_state_dict(sd)
        if step == 10:
            for m in (eager, rep):
                sd = m.opt_D.state_dict()
                for st in sd["state"].values():
                    st["step"] = torch.tensor(float(m.fpD.step - 2))
                m.opt_D.load_state_dict(sd)
        n0 = rep.graph_replays
        eager.train_step()
        rep.train_step()
        replayed += rep.graph_replays - n0
        torch.cuda.synchronize()
        a, b = state(eager), state(rep)
        assert eager.fpG.step == rep.fpG.step == step + 1
        assert int(rep.fpD.step_dev.item()) == rep.fpD.step
        for k in a:
            assert torch.equal(a[k], b[k]), (step, k, float((a[k].double() - b[k].double()).abs().max()))
        assert rep.graph_replays - n0 == (1 if step in (3, 4, 5) else 0), step
    assert replayed == 3, replayed
    rec = rep._gstate.get("rec")
    assert rec is not None and len(rec) > 50, "recording holds the step's launches"


@pytest.mark.parametrize("dtype", ["bf16"])
def test_cpp_replay_under_dp_exchange_bitwise(tmp_path, dtype):
    """The C++ replay with the DP exchange on (an RCCL group of one rank, the bench's
    --dp-exchange): the exchange's collectives, seals and waits are host actions recorded
    between the launch segments (dp.GradExchange._act), the G exchange deferred across the
    step boundary (the second-backward reorder) -- against the same model stepped eagerly:
    BITWISE equal after every step, with replays from the fourth step on.  flush() (what
    save_checkpoint does, on rank 0 only in train.py) runs between steps four times at the same
    key: the steps after a flush start with no deferred G update (the other recording), and a
    replay must leave the engine's deferred-update state where the recorded step left it, or
    the next step re-replays the no-pending recording and Adam_G never runs again."""
    import torch.distributed as dist
    from test_gpu_dp import _free_port
    if not dist.is_initialized():
        import os
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(_free_port())
        dist.init_process_group("nccl", rank=0, world_size=1)
        own = True
    else:
        own = False
    try:
        args = make_args(tmp_path, depths=list(TINY_DEPTHS), compute_dtype=dtype)
        args.update({"dp_exchange_world1": True})
        s = 3
        eager, rep = build(args, False, s), build_replay(args, s)
        for m in (eager, rep):
            m.set_multi_GPU()
            m.G.alpha = m.D.alpha = 0.5
        replayed = 0
        for step in range(16):
            n0 = rep.graph_replays
            eager.train_step()
            rep.train_step()
            replayed += rep.graph_replays - n0
            if step in (6, 8, 10, 12, 15):
                for m in (eager, rep):
                    m.flush()
            torch.cuda.synchronize()
            a, b = state(eager), state(rep)
            for k in a:
                assert torch.equal(a[k], b[k]), (step, k, float((a[k].double() - b[k].double()).abs().max()))
            ee, er = (next(iter(m._engines.values())) for m in (eager, rep))
            assert (ee._pending_G is None) == (er._pending_G is None), step
            assert eager.fpG.step == rep.fpG.step, step
        assert int(rep.fpG.step_dev.item()) == rep.fpG.step
        assert replayed >= 8, replayed
        assert rep._exchange.calls > 0
    finally:
        if own:
            dist.destroy_process_group()
