"""CPU tests of the C-ABI boundary: the library loads, exports every symbol include/gptsgld.h
declares, and its host-only entry points (no device work) agree with the oracle exactly."""
import os
import re

import numpy as np
import pytest

from oracle import gpt_sgld_ref as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "gptsgld.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?(?:int|void|int64_t|char\s*\*|const char\s*\*)\s*\**\s*(gpt_\w+)\s*\(",
                       txt, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = header_functions()
    for want in ["gpt_feature", "gpt_feature_notensor", "gpt_samplenz", "gpt_sgld_regression",
                 "gpt_pred", "gpt_pred_mean", "gpt_gpnt_sgld", "gpt_last_error",
                 "gpt_sgld_session_create", "gpt_sgld_session_run"]:
        assert want in names


def test_library_exports_every_header_symbol():
    from gpt_amd import _lib
    lib = _lib.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, name


def test_samplenz_host_matches_oracle():
    from gpt_amd import GPT_SGLD as G
    for (r, D, Q, s) in [(5, 8, 200, 17), (2, 5, 32, 3), (20, 8, 200, 1), (3, 3, 27, 2)]:
        assert (G.samplenz(r, D, Q, s) == R.samplenz(r, D, Q, s)).all()


def test_init_state_host_matches_oracle():
    from gpt_amd import GPT_SGLD as G
    for stf in (True, False):
        w, U = G.init_state(60, 5, 3, 40, 77, stiefel=stf)
        wo, Uo = R.init_state(60, 5, 3, 40, 77, stiefel=stf)
        assert np.abs(w - wo).max() == 0.0
        assert np.abs(U - Uo).max() < 1e-14


def test_feature_inputs_host_matches_oracle():
    from gpt_amd import GPT_SGLD as G
    Z, b = G.feature_inputs(30, 6, 17)
    Zo, bo = R.seeded_feature_inputs(30, 6, 17)
    assert np.abs(Z - Zo).max() < 1e-15 and np.abs(b - bo).max() < 1e-15


def test_feature_inputs_generation_a_host_matches_oracle():
    """Gen A (GPT_SGLD_p.jl:43-45): b = randn(n,D), not 2π·rand."""
    from gpt_amd import GPT_SGLD as G
    Z, b = G.feature_inputs_a(30, 6, 17)
    Zo, bo = R.seeded_feature_inputs_a(30, 6, 17)
    assert np.abs(Z - Zo).max() < 1e-15 and np.abs(b - bo).max() < 1e-15
    assert b.min() < 0.0                                   # normal, not uniform on [0, 2π)
    Zc, _ = G.feature_inputs(30, 6, 17)
    assert np.array_equal(Z, Zc)                           # the Z stream is shared with Gen C


def test_bad_arguments_fail_without_device():
    from gpt_amd import GPT_SGLD as G
    from gpt_amd._lib import GPTError
    with pytest.raises(GPTError):
        G.samplenz(2, 3, 9, 0)          # Q > r^D
