"""gpt_amd — MI355X-native (HIP/gfx950) tensor-GP SGLD path of hyunjik11/GPT.

``gpt_amd.GPT_SGLD`` mirrors the reference's Julia module API over libgptsgld.so;
``gpt_amd.TGP`` mirrors the ``TGP`` module (Gibbs sampler, TGP.jl);
``gpt_amd.session`` drives device-resident multi-chain runs (benchmark / multi-GPU).
"""
from . import _lib  # noqa: F401  (loads nothing until first use)

__all__ = ["GPT_SGLD", "TGP", "session"]
