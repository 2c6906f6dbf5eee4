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
kus = bench.gather_over_ranks(90.0 + rank)     # per-rank kernel time in the line
seeds = bench.chain_seeds(rank, 1000)
with open(os.path.join(%r, "rank%%d.json" %% rank), "w") as f:
    json.dump(dict(rank=rank, world=dist.get_world_size(), local=int(os.environ["LOCAL_RANK"]),
                   dt=dt, argv=sys.argv[1:], kus=kus, seeds=seeds), f)
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
    assert all(g["kus"] == [90.0, 91.0] for g in got)
    # 1000 chains per rank: the seeds of the two ranks do not collide (round-2 seeds did)
    assert len(set(got[0]["seeds"]) | set(got[1]["seeds"])) == 2000


def test_chain_seeds_distinct_over_ranks():
    import bench
    for C in (1, 7, 256, 1000, 1024):
        allseeds = [s for rk in range(8) for s in bench.chain_seeds(rk, C)]
        scratch = [s for rk in range(8) for s in bench.scratch_seeds(rk, C)]
        assert len(set(allseeds)) == 8 * C and len(set(scratch)) == 8 * C
        assert not set(allseeds) & set(scratch)


def test_bench_line_fields_at_world_2():
    """The rank-0 line of an N = 2 run carries the same fields as N = 1: cpu_baseline, per-rank
    kernel times, the single-chain pass (a SCALE line has what a BENCH line has)."""
    import types
    import bench
    args = types.SimpleNamespace(workload="kin40k", steps=20, warmup=5, epsw=1e-5, epsU=1e-8,
                                 signal_var=0.0476)
    quality = dict(test_rmse=0.28, note="x")
    common = dict(args=args, value=5.0e6, warm_ms=300.0, dataset="kin40k", ms_per_step=0.1, wdesc="kin40k", N=10000,
                  Nte=30000, D=8, n=500, r=5, Q=200, m=50, C=256, alive=256,
                  info=dict(engine="chain", workgroups=256, threads=512, lds_bytes=73600),
                  roof={"bound": "hbm", "achieved": 5000.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.625}, traffic=4.2e8, traffic_src="t", bytes_launch=4.94e8,
                  steps_run=41000, cpu=dict(value=17000.0, cores=16, kind="port"),
                  quality=quality, allreduce_ms=0.05, npred=256, pred_ms=6.9, pred_flop=3.07e11,
                  gemm_ms=5.4, vphase_ms=1.0, rmse_final=0.28,
                  vphase_kernel="pred_vphase_pairs_kernel", host_us={},
                  single=dict(steps_per_s=2e4, kernel_us=50.0))
    one = bench.compose_line(types.SimpleNamespace(world=1, world_seen=1, k_us=93.0,
                                                   k_us_ranks=[93.0], **common))
    two = bench.compose_line(types.SimpleNamespace(world=2, world_seen=2, k_us=93.0,
                                                   k_us_ranks=[93.0, 94.0], **common))
    assert set(one) == set(two) and set(one["roofline"]) == set(two["roofline"])
    assert two["n_gpus"] == 2 and two["cpu_baseline"]["cores"] == 16
    assert two["roofline"]["kernel_us_per_rank"] == [93.0, 94.0]
    assert two["single_chain"]["steps_per_s"] == 2e4
    assert two["config"]["parallelism"] == "chains256x2"
    assert "tests/golden/kin40k.npz" in two["data"]
    assert two["pred"]["kernels"].endswith("pred_vphase_pairs_kernel")
