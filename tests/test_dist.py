"""Multi-rank sharding on CPU: world_size 2 (and 3) over gloo.

Each rank renders its interleaved stripe set exactly as a GPU rank does
(rt_dispatch_rows' mapping, here through the oracle), the buffers fan in to
rank 0 with tiling.gather_to_root, and the reassembled frame must equal the
single-process frame bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import rtamd
import tiling


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, stripe, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fs = rtamd.generate(2, 0, W, H)
        plan = tiling.StripePlan(H, world, stripe)
        local = torch.zeros((plan.rows_max, W, 4), dtype=torch.float32)
        n = plan.rows(rank)
        if n:
            img, _ = oracle.render(fs, W, H, oracle.params(W, H, 1), y0=plan.y0(rank), stripe=stripe, step=world,
                                   out_rows=n)
            local[:n] = torch.from_numpy(img)
        full = tiling.gather_to_root(local, plan)
        if rank == 0:
            np.save(out_path, full.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,stripe,H", [(2, 8, 48), (3, 8, 50), (2, 4, 13)])
def test_stripe_gather_matches_single_frame(tmp_path, world, stripe, H):
    W = 40
    out = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, stripe, out), nprocs=world, join=True)
    got = np.load(out)
    fs = rtamd.generate(2, 0, W, H)
    ref, _ = oracle.render(fs, W, H, oracle.params(W, H, 1))
    assert np.array_equal(got, ref)


def test_stripe_plan_covers_every_row_once():
    for H in (1, 7, 8, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            plan = tiling.StripePlan(H, world, 8)
            rows = torch.cat([plan.image_rows(r) for r in range(world)])
            assert sorted(rows.tolist()) == list(range(H))


def test_root_share_plan_covers_every_row_once():
    """rt_group's rows with rank 0 taking `share` stripes per period (SharePlan
    restates csrc/rt_group.hip rank_rows): every image row once; share 1 is the
    plain interleave; rank 1 holds the most rows of ranks >= 1 (its count sizes
    the staging slots)."""
    for H in (1, 7, 8, 13, 270, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            for share in (1, 2, 3):
                for stripe in (1, 3, 8):
                    plan = tiling.SharePlan(H, world, stripe, share)
                    rows = torch.cat([plan.image_rows(r) for r in range(world)])
                    assert sorted(rows.tolist()) == list(range(H)), (H, world, share, stripe)
                    n = [plan.mapping(r)[3] for r in range(world)]
                    assert all(n[1] >= x for x in n[1:]) if world > 1 else True
                    if share == 1:
                        sp = tiling.StripePlan(H, world, stripe)
                        assert all(torch.equal(plan.image_rows(r), sp.image_rows(r)) for r in range(world))
    # at 1080p over 2 GPUs, share 2 leaves rank 1 a third of the rows to send instead of half
    assert tiling.SharePlan(1080, 2, 8, 2).mapping(1)[3] == 360
