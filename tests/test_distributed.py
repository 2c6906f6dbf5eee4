"""World-size-2 gloo test of the multi-GPU combine (the path's single collective)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpt_amd.ensemble import combine_predictive_mean
    rng = np.random.default_rng(rank)
    k = 3 + rank                                   # ranks may hold different sample counts
    preds = rng.standard_normal((k, 17))
    fsum = torch.from_numpy(preds.sum(axis=0).copy())
    mean = combine_predictive_mean(fsum, k)
    out[rank] = mean.numpy()
    dist.destroy_process_group()


def test_gloo_world2_predictive_mean():
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    allp = np.concatenate([np.random.default_rng(r).standard_normal((3 + r, 17)) for r in range(world)])
    want = allp.mean(axis=0)
    for r in range(world):
        assert np.allclose(out[r], want, rtol=1e-14, atol=1e-14)


def test_single_process_combine_is_identity_mean():
    from gpt_amd.ensemble import combine_predictive_mean, rmse
    f = torch.tensor([2.0, 4.0, 6.0], dtype=torch.float64)
    assert torch.allclose(combine_predictive_mean(f.clone(), 2), f / 2)
    assert rmse([1.0, 2.0, 3.0], [1.0, 2.0, 3.0]) == 0.0
