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


_RANK_SCRIPT = """
import json, os, sys, time
sys.path.insert(0, %r)
import torch.distributed as dist
import bench
dist.init_process_group("gloo")
rank = dist.get_rank()
dt = bench.max_over_ranks(0.5 + rank)          # rank r 'took' 0.5 + r seconds
with open(os.path.join(%r, "rank%%d.json" %% rank), "w") as f:
    json.dump(dict(rank=rank, world=dist.get_world_size(), local=int(os.environ["LOCAL_RANK"]),
                   dt=dt, argv=sys.argv[1:]), f)
dist.destroy_process_group()
"""


def test_bench_launcher_command():
    import bench
    cmd = bench.launch_command(["--gpus", "8", "--steps", "20"], 8, 29511)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "20"] and cmd[-5].endswith("bench.py")


def test_bench_self_launch_gloo_world2(tmp_path):
    """bench.self_launch starts N ranks (a child torchrun, as `python bench.py --gpus N` does when
    WORLD_SIZE is unset); every rank sees world size N and the max-over-ranks timing."""
    import bench
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "rank_script.py"
    script.write_text(_RANK_SCRIPT % (root, str(tmp_path)))
    env_keep = {k: os.environ.pop(k) for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK") if k in os.environ}
    try:
        rc = bench.self_launch(["--steps", "3"], 2, script=str(script))
    finally:
        os.environ.update(env_keep)
    assert rc == 0
    import json
    got = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(2)]
    assert sorted(g["rank"] for g in got) == [0, 1]
    assert all(g["world"] == 2 and g["dt"] == 1.5 and g["argv"] == ["--steps", "3"] for g in got)
    assert sorted(g["local"] for g in got) == [0, 1]
