"""Multi-GPU combine of independent chains: the only collective of the path.

Each rank runs its own chains with no data-path communication; at the end (or per epoch) the ranks
sum their per-rank predictive-mean vectors with one all-reduce (RCCL over xGMI on the GPU box, gloo in
the CPU tests) — the ``@parallel (+)`` reduction of ``RMSE`` (GPT_SGLD_p.jl:124-132).
"""
import math

import numpy as np


def combine_predictive_mean(fsum, count, group=None):
    """fsum: this rank's sum of per-sample predictions (torch tensor, Ntest); count: how many
    samples it summed.  Returns the posterior-mean prediction over all ranks' samples."""
    import torch
    import torch.distributed as dist
    n = torch.tensor([float(count)], dtype=fsum.dtype, device=fsum.device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(fsum, group=group)
        dist.all_reduce(n, group=group)
    return fsum / n


def rmse(ytest, fmean, scale=1.0):
    """kin40kExperiment.jl:83 — scale·‖ytest − fmean‖/sqrt(Ntest)."""
    ytest = np.asarray(ytest, dtype=np.float64).ravel()
    fmean = np.asarray(fmean, dtype=np.float64).ravel()
    return float(scale * np.linalg.norm(ytest - fmean) / math.sqrt(len(ytest)))
