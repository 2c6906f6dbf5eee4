"""ctypes binding of libgptsgld.so (include/gptsgld.h).

This is the product path: every call goes through the HIP library.  There is no CPU
fallback — if the shared object is missing the import fails loudly.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPTSGLD_LIB") or os.path.join(_HERE, "libgptsgld.so")

GPT_OK = 0
GPT_ERR_NAN_GEODESIC = 1
GPT_ERR_BAD_DIMS = 2
GPT_ERR_HIP = 3
GPT_ERR_NAN_THETA = 4
GPT_ERR_NOT_SPD = 5

P_D = C.POINTER(C.c_double)
P_I32 = C.POINTER(C.c_int32)
P_U64 = C.POINTER(C.c_uint64)


class SGLDConfig(C.Structure):
    """Mirror of ``gpt_sgld_config`` (include/gptsgld.h)."""
    _fields_ = [("n", C.c_int64), ("D", C.c_int64), ("N", C.c_int64), ("r", C.c_int64),
                ("Q", C.c_int64), ("m", C.c_int64), ("epsw", C.c_double), ("epsU", C.c_double),
                ("signal_var", C.c_double), ("sigma_w", C.c_double), ("burnin", C.c_int64),
                ("maxepoch", C.c_int64), ("seed", C.c_uint64), ("langevin", C.c_int32),
                ("stiefel", C.c_int32), ("store_every", C.c_int64), ("max_steps", C.c_int64)]


# name -> (restype, argtypes)
SIGNATURES = {
    "gpt_feature": (C.c_int, [P_D, C.c_int64, C.c_int64, P_D, C.c_int64, C.c_double, C.c_double,
                              P_D, P_D, C.c_int64, P_D]),
    "gpt_feature_notensor": (C.c_int, [P_D, C.c_int64, C.c_int64, P_D, C.c_int64, C.c_double,
                                       P_D, P_D, C.c_int64, P_D]),
    "gpt_feature_inputs": (C.c_int, [C.c_int64, C.c_int64, C.c_uint64, P_D, P_D]),
    "gpt_feature_inputs_a": (C.c_int, [C.c_int64, C.c_int64, C.c_uint64, P_D, P_D]),
    "gpt_epoch_orders": (C.c_int, [C.c_int64, C.c_uint64, C.c_int64, P_I32]),
    "gpt_samplenz": (C.c_int, [C.c_int64, C.c_int64, C.c_int64, C.c_uint64, P_I32]),
    "gpt_sgld_init": (C.c_int, [C.POINTER(SGLDConfig), P_D, P_D]),
    "gpt_sgld_regression": (C.c_int, [C.POINTER(SGLDConfig), P_D, P_D, P_I32, P_D, P_D, P_D, P_D,
                                      P_D]),
    "gpt_sgld_regression_chains": (C.c_int, [C.POINTER(SGLDConfig), C.c_int32, P_U64,
                                             C.POINTER(P_D), C.POINTER(P_D), P_I32, P_D, P_D, P_D,
                                             C.POINTER(P_D), C.POINTER(P_D), P_I32]),
    "gpt_sgld_session_create": (C.c_int, [C.POINTER(SGLDConfig), C.c_int32, P_U64,
                                          C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), P_I32,
                                          C.c_int32, C.c_void_p, C.POINTER(C.c_void_p)]),
    "gpt_sgld_session_run": (C.c_int, [C.c_void_p, C.c_int64]),
    "gpt_sgld_session_prepare": (C.c_int, [C.c_void_p, C.c_int64]),
    "gpt_sgld_session_set_rmsprop": (C.c_int, [C.c_void_p, C.c_double, C.c_double]),
    "gpt_sgld_rmsprop": (C.c_int, [C.POINTER(SGLDConfig), C.c_double, C.c_double, P_D, P_D, P_I32,
                                   P_D, P_D, P_D, P_D, P_D]),
    "gpt_sgld_session_set_hyper": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_double,
                                             C.c_double, C.c_double]),
    "gpt_sgld_session_sync": (C.c_int, [C.c_void_p]),
    "gpt_sgld_session_state": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]),
    "gpt_sgld_session_gather_state": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                                                C.c_void_p]),
    "gpt_sgld_session_steps_done": (C.c_int64, [C.c_void_p]),
    "gpt_sgld_session_time_steps": (C.c_int, [C.c_void_p, C.c_int64, P_D]),
    "gpt_sgld_session_stamps": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
    "gpt_sgld_timeline_slots": (C.c_int64, []),
    "gpt_debug_expm_stamps": (C.c_int, [C.c_int32, C.c_int32, P_D, C.POINTER(C.c_int64)]),
    "gpt_debug_expm": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, P_D, P_D, P_I32]),
    "gpt_debug_gaussian_draw": (C.c_int, [C.c_int32, P_D, P_D, C.c_uint64, C.c_uint32, C.c_uint32,
                                          C.c_uint32, P_D, P_I32]),
    "gpt_pred_trim_pool": (C.c_int, []),
    "gpt_cf_last_timing": (C.c_int, [P_D, P_D, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "gpt_cf_last_mode": (C.c_int, [C.POINTER(C.c_int32)]),
    "gpt_pred_last_vphase": (C.c_int, [C.POINTER(C.c_int32)]),
    "gpt_cf_last_stamps": (C.c_int64, [C.POINTER(C.c_int64), C.c_int64]),
    "gpt_sgld_session_timeline": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(C.c_int64), P_D]),
    "gpt_feature_dev": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64,
                                  C.c_double, C.c_double, C.c_void_p, C.c_void_p, C.c_int64,
                                  C.c_void_p, C.c_void_p]),
    "gpt_sgld_session_fetch": (C.c_int, [C.c_void_p, C.c_int32, P_D, P_D, P_D, P_I32]),
    "gpt_sgld_session_destroy": (None, [C.c_void_p]),
    "gpt_sgld_session_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "gpt_pred": (C.c_int, [P_D, P_D, P_I32, P_D, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                           C.c_int64, P_D]),
    "gpt_pred_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                               C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_void_p,
                               C.c_void_p]),
    "gpt_pred_dev_timed": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                     C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                     C.c_void_p, C.c_void_p, P_D]),
    "gpt_pred_mean": (C.c_int, [P_D, P_D, P_I32, P_D, P_D, C.c_int64, C.c_int64, C.c_int64,
                                C.c_int64, C.c_int64, C.c_int64, C.c_double, P_D, P_D]),
    "gpt_gpnt_sgld": (C.c_int, [P_D, P_D, C.c_int64, C.c_int64, C.c_double, C.c_double, C.c_int64,
                                C.c_double, C.c_double, C.c_int64, C.c_int64, C.c_uint64, P_D]),
    "gpt_sgld_wonly": (C.c_int, [C.POINTER(SGLDConfig), P_D, P_D, P_I32, P_D, P_D, P_D, P_D, P_D]),
    "gpt_pred_mean_x": (C.c_int, [P_D, P_D, P_I32, P_D, P_D, C.c_int64, C.c_int64, P_D, C.c_int64,
                                  C.c_double, C.c_double, P_D, P_D, C.c_int64, C.c_int64, C.c_int64,
                                  C.c_int64, C.c_double, P_D, P_D, P_D]),
    "gpt_sgld_classification": (C.c_int, [C.POINTER(SGLDConfig), P_D, P_D, P_I32, P_D, P_D, P_D,
                                          P_D, P_D]),
    "gpt_gmc": (C.c_int, [P_D, P_D, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64, P_I32,
                          C.c_double, C.c_double, C.c_double, C.c_int64, C.c_int64, C.c_int64,
                          C.c_uint64, P_D, P_D, P_D, P_D, P_D]),
    "gpt_cf_fullw_sideinfo": (C.c_int, [P_D, C.c_int64, C.c_int64, P_D, C.c_int64, C.c_int64, P_D,
                                        C.c_int64, C.c_int64, P_D, C.c_int64, C.c_int64,
                                        C.c_double, C.c_double, C.c_double, P_D, C.c_int64,
                                        C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double,
                                        C.c_double, C.c_int64, C.c_int64, C.c_uint64, C.c_double,
                                        C.c_double, C.c_int32, C.c_int32, C.c_int32, P_D, P_D, P_D,
                                        P_D, P_D, P_D]),
    "gpt_cf_fullw_gibbs": (C.c_int, [P_D, C.c_int64, C.c_int64, C.c_int64, C.c_int64, P_D, C.c_int64,
                                     C.c_int64, C.c_double, C.c_double, C.c_double, P_D, C.c_int64,
                                     C.c_int64, C.c_int64, C.c_int64, C.c_uint64, C.c_double,
                                     C.c_double, C.c_int32, C.c_int32, P_D, P_D, P_D, P_D, P_D,
                                     P_D]),
    "gpt_cf_fullw_sideinfo_folds": (C.c_int, [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_void_p, P_D, C.c_int64, C.c_int64, P_D,
                                              C.c_int64, C.c_int64, C.c_double, C.c_double,
                                              C.c_double, P_D, C.c_int64, C.c_int64, C.c_double,
                                              C.c_double, C.c_double, C.c_double, C.c_double,
                                              C.c_int64, C.c_int64, C.c_uint64, P_D, P_D,
                                              C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_void_p, P_I32]),
    "gpt_cf_fixw_sideinfo": (C.c_int, [P_D, C.c_int64, C.c_int64, P_D, C.c_int64, C.c_int64, P_D,
                                       C.c_int64, C.c_int64, P_D, C.c_int64, C.c_int64,
                                       C.c_double, C.c_double, P_D, C.c_int64, C.c_int64,
                                       C.c_double, C.c_double, C.c_double, C.c_double, C.c_int64,
                                       C.c_int64, C.c_uint64, C.c_double, C.c_double, C.c_int32,
                                       C.c_int32, C.c_int32, P_D, P_D, P_D, P_D, P_D]),
    "gpt_cf_fullw": (C.c_int, [P_D, C.c_int64, C.c_int64, C.c_int64, C.c_int64, P_D, C.c_int64,
                               C.c_int64, C.c_double, C.c_double, C.c_double, P_D, C.c_int64,
                               C.c_int64, C.c_double, C.c_double, C.c_int64, C.c_int64,
                               C.c_uint64, C.c_double, C.c_double, C.c_int32, C.c_int32,
                               C.c_int32, P_D, P_D, P_D, P_D, P_D, P_D]),
    "gpt_cf_fixw": (C.c_int, [P_D, C.c_int64, C.c_int64, C.c_int64, C.c_int64, P_D, C.c_int64,
                              C.c_int64, C.c_double, C.c_double, P_D, C.c_int64, C.c_int64,
                              C.c_double, C.c_int64, C.c_int64, C.c_uint64, C.c_double, C.c_double,
                              C.c_int32, C.c_int32, C.c_int32, P_D, P_D, P_D, P_D, P_D]),
    "gpt_cf_fixw_gibbs": (C.c_int, [P_D, C.c_int64, C.c_int64, C.c_int64, C.c_int64, P_D,
                                    C.c_int64, C.c_int64, C.c_double, C.c_double, P_D, C.c_int64,
                                    C.c_int64, C.c_int64, C.c_int64, C.c_uint64, C.c_double,
                                    C.c_double, C.c_int32, C.c_int32, P_D, P_D, P_D, P_D, P_D]),
    "gpt_tgp_gibbs": (C.c_int, [P_D, P_D, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                C.c_double, C.c_int64, C.c_int64, C.c_uint64, P_I32, P_D, P_D,
                                P_I32]),
    "gpt_last_error": (C.c_char_p, []),
    "gpt_sgld_lds_bytes": (C.c_int64, [C.c_int64] * 5),
    "gpt_device_count": (C.c_int, []),
}


def load(path=LIB_PATH):
    # Bind to the HIP runtime torch already carries (one runtime per process): torch's
    # bundled libamdhip64 has the same soname, so loading torch first makes the dynamic
    # loader resolve our NEEDED entry to it instead of pulling in a second runtime.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(path):
        raise ImportError(
            "libgptsgld.so not found at %s — build it with `python -c \"import __graft_entry__ as g; "
            "g.build()\"` (hipcc --offload-arch=gfx950). There is no CPU fallback." % path)
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None and path != os.path.join(_HERE, "libgptsgld.so"):
            continue          # an older comparison build named by GPTSGLD_LIB (A/B runs)
        if fn is None:
            raise ImportError("%s does not export %s: rebuild it" % (path, name))
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = load()
    return _LIB


class GPTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("gptsgld error %d: %s" % (code, msg))
        self.code = code


def check(code):
    if code != GPT_OK:
        raise GPTError(code, lib().gpt_last_error().decode(errors="replace"))
    return code
