"""The Julia ccall shims (julia/*.jl) against the C prototypes of include/gptsgld.h.

Julia is not on the image, so the shims cannot run here.  This test parses every
`ccall((:sym, LIB), RetT, (ArgT, ...), args...)` and checks the symbol exists in the header, the
argument count matches the prototype and every Julia type is the one the C type needs; it also
checks the SGLDConfig mirror against `gpt_sgld_config`, and that every entry point INTEGRATION.md
lists has a Julia binding.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JULIA = [os.path.join(ROOT, "julia", f) for f in ("GPT_SGLD_HIP.jl", "MovieLens_HIP.jl", "TGP_HIP.jl")]

# C type (normalised) -> accepted Julia ccall types
C2J = {
    "int": {"Cint", "Int32"},
    "int32_t": {"Int32", "Cint"},
    "int64_t": {"Int64"},
    "uint64_t": {"UInt64"},
    "double": {"Float64", "Cdouble"},
    "void": {"Cvoid", "Nothing"},
    "const char*": {"Cstring", "Ptr{UInt8}"},
    "double*": {"Ptr{Float64}", "Ref{Float64}"},
    "const double*": {"Ptr{Float64}"},
    "int32_t*": {"Ptr{Int32}"},
    "const int32_t*": {"Ptr{Int32}"},
    "const int64_t*": {"Ptr{Int64}"},
    "const uint64_t*": {"Ptr{UInt64}"},
    "const double* const*": {"Ptr{Ptr{Float64}}"},
    "double* const*": {"Ptr{Ptr{Float64}}"},
    "const gpt_sgld_config*": {"Ref{SGLDConfig}", "Ptr{SGLDConfig}"},
    "gpt_sgld_session*": {"Ptr{Cvoid}"},
    "void*": {"Ptr{Cvoid}"},
}


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", " ", re.sub(r"//[^\n]*", " ", s, flags=re.S), flags=re.S)


def _norm_ctype(t):
    t = re.sub(r"\s+", " ", t.strip())
    t = re.sub(r"\s*\*\s*", "*", t)
    t = t.replace("*const*", "* const*")
    return t


def header_prototypes():
    src = _strip_c_comments(open(os.path.join(ROOT, "include", "gptsgld.h")).read())
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(gpt_\w+)\s*\(([^;{]*?)\)\s*;", src):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        ret = _norm_ctype(ret.replace("typedef", ""))
        params = []
        if args.strip() not in ("", "void"):
            for a in args.split(","):
                a = a.strip()
                mm = re.match(r"(.*?)(\w+)$", a)           # drop the parameter name
                params.append(_norm_ctype(mm.group(1)))
        protos[name] = (ret, params)
    return protos


def _split_top(s):
    """Split s at commas of bracket depth 0."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _balanced(s, i):
    """Index just past the bracket group opening at s[i]."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] in "({[":
            depth += 1
        elif s[j] in ")}]":
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced")


def julia_ccalls(path):
    src = re.sub(r"#[^\n]*", "", open(path).read())
    calls = []
    for m in re.finditer(r"ccall\(\(:(\w+),\s*LIB\),\s*", src):
        start = m.end()
        # return type up to the comma at depth 0
        j, depth = start, 0
        while not (src[j] == "," and depth == 0):
            depth += src[j] in "({[" and 1 or 0
            depth -= src[j] in ")}]" and 1 or 0
            j += 1
        ret = src[start:j].strip()
        k = j + 1
        while src[k].isspace():
            k += 1
        assert src[k] == "(", (m.group(1), src[k:k + 20])
        e = _balanced(src, k)
        types = _split_top(src[k + 1:e - 1])
        # the call's own argument list: from after the types tuple to the ccall's closing paren
        open_paren = m.start() + len("ccall")
        close = _balanced(src, open_paren)
        rest = src[e:close - 1].strip()
        args = _split_top(rest[1:]) if rest.startswith(",") else []
        calls.append((m.group(1), ret, types, args))
    return calls


def all_calls():
    out = []
    for p in JULIA:
        out += [(os.path.basename(p),) + c for c in julia_ccalls(p)]
    return out


def test_every_ccall_matches_the_header():
    protos = header_prototypes()
    calls = all_calls()
    assert len(calls) >= 25
    for fname, sym, ret, types, args in calls:
        assert sym in protos, "%s: %s is not declared in include/gptsgld.h" % (fname, sym)
        cret, cparams = protos[sym]
        assert ret in C2J[cret], "%s: %s returns %s, C returns %s" % (fname, sym, ret, cret)
        assert len(types) == len(cparams), "%s: %s has %d argument types, C has %d" % (
            fname, sym, len(types), len(cparams))
        assert len(args) == len(types), "%s: %s passes %d arguments for %d types" % (
            fname, sym, len(args), len(types))
        for i, (jt, ct) in enumerate(zip(types, cparams)):
            assert ct in C2J, "unmapped C type %r (%s arg %d)" % (ct, sym, i)
            assert jt in C2J[ct], "%s: %s arg %d is %s, C wants %s" % (fname, sym, i, jt, ct)


def test_sgld_config_mirror_matches_the_header():
    src = _strip_c_comments(open(os.path.join(ROOT, "include", "gptsgld.h")).read())
    body = re.search(r"typedef struct gpt_sgld_config \{(.*?)\} gpt_sgld_config;", src, re.S).group(1)
    cfields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        t, names = re.match(r"(\w+)\s+(.*)", decl).groups()
        cfields += [(n.strip(), t) for n in names.split(",")]
    jsrc = open(JULIA[0]).read()
    jbody = re.search(r"struct SGLDConfig.*?\n(.*?)\nend", jsrc, re.S).group(1)
    jfields = []
    for decl in re.sub(r"#[^\n]*", "", jbody).replace("\n", ";").split(";"):
        decl = decl.strip()
        if decl:
            n, t = decl.split("::")
            jfields.append((n.strip(), t.strip()))
    cmap = {"int64_t": "Int64", "double": "Float64", "uint64_t": "UInt64", "int32_t": "Int32"}
    assert [(n, cmap[t]) for n, t in cfields] == jfields


def test_integration_entry_points_have_julia_bindings():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    table = text.split("## Julia")[0]
    listed = set(re.findall(r"`(gpt_\w+)`", table))
    bound = {c[1] for c in all_calls()}
    # device-resident / session entry points take device pointers or torch-owned streams: they are
    # the Python/C++ host's interface (the Julia host calls the host-pointer forms)
    device_only = {s for s in listed if s.endswith("_dev") or s.startswith("gpt_sgld_session")}
    missing = sorted(listed - device_only - bound)
    assert not missing, "INTEGRATION.md entry points without a Julia binding: %s" % missing


@pytest.mark.parametrize("sym", ["gpt_cf_fixw", "gpt_cf_fullw", "gpt_cf_fixw_sideinfo",
                                 "gpt_cf_fixw_gibbs", "gpt_cf_fullw_sideinfo_folds",
                                 "gpt_feature_inputs", "gpt_pred_mean_x", "gpt_sgld_init",
                                 "gpt_sgld_regression_chains"])
def test_round3_bindings_present(sym):
    assert sym in {c[1] for c in all_calls()}
