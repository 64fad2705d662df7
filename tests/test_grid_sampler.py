"""Image-grid layout and the per-rank sample order against restatements of the reference's
helpers: torchvision.utils.make_grid as lib/utils.py:94-103 calls it, and
torch.utils.data.DistributedSampler as lib/model.py:50 builds it (torchvision is not
installed here; DistributedSampler is torch's own and is run directly)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from pggan_amd.model import make_grid_image, sampler_order


def grid_restated(list_of_tensors):
    """make_grid(nrow = n, padding = 2, pad_value = 0) per row, * 0.5 + 0.5, rows stacked:
    every image framed by F.pad on its top/left, one extra 2-px strip on the bottom/right."""
    rows = []
    for t in list_of_tensors:
        t = t[:8].float()
        if t.shape[0] == 1:
            rows.append(t[0] * 0.5 + 0.5)
            continue
        tiles = [F.pad(im, (2, 0, 2, 0)) for im in t]
        row = torch.cat(tiles, dim=2)
        row = F.pad(row, (0, 2, 0, 2))
        rows.append(row * 0.5 + 0.5)
    return torch.cat(rows, dim=1)


@pytest.mark.parametrize("n", [1, 3, 8, 11])
def test_make_grid_layout(n):
    g = torch.Generator().manual_seed(n)
    a = torch.rand(n, 3, 16, 16, generator=g) * 2.4 - 1.2   # values past [-1, 1] stay
    b = torch.rand(n, 3, 16, 16, generator=g) * 2 - 1
    got = make_grid_image([a, b])
    want = grid_restated([a, b])
    assert got.shape == want.shape
    assert torch.equal(got, want)
    if n > 1:
        k = min(n, 8)
        assert got.shape == (3, 2 * (16 + 2 + 2), k * 18 + 2)   # two rows, 2-px frames
        assert float(got[0, 0, 0]) == 0.5                    # padding 0 -> 0.5 after * .5 + .5


@pytest.mark.parametrize("n,world", [(10, 1), (10, 2), (11, 4), (3, 8), (1000, 8)])
def test_sampler_order_matches_distributed_sampler(n, world):
    ds = list(range(n))
    for rank in range(world):
        got = sampler_order(n, rank, world)
        if world == 1:
            want = np.arange(n)    # no sampler in one process: DataLoader order
        else:
            s = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=world,
                                                                rank=rank)
            want = np.asarray(list(iter(s)))
        assert np.array_equal(got, want), (rank, got[:8], want[:8])
        assert len(got) == (n if world == 1 else math.ceil(n / world))


@pytest.mark.parametrize("n", [10, 7])
def test_sampler_order_use_mgpu_one_rank(n):
    """use_mGPU with gpu_num = 1: the reference still builds a DistributedSampler (shuffled)."""
    s = torch.utils.data.distributed.DistributedSampler(list(range(n)), num_replicas=1, rank=0)
    assert np.array_equal(sampler_order(n, 0, 1, distributed=True), np.asarray(list(iter(s))))
    assert np.array_equal(sampler_order(n, 0, 1, distributed=False), np.arange(n))
