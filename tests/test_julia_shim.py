"""Static check of the Julia drop-in shim (torj.jl_amd/julia/TorJHIP.jl) against
the C header (include/torj_hip.h) -- the only guard possible without a Julia
toolchain in this container or on the GPU box.

Every `ccall((:sym, libtorj), Ret, (Types...), args...)` in the shim must name a
symbol the library exports and the header declares, with the same return type,
the same number of arguments (types and actual arguments alike) and matching
types position by position; the shim's `TraceCfg` must list the C struct's
fields in order with matching types.  The reference signatures the shim
reproduces are TorJ.jl src/solve.jl:135-136 (make_ray) and :209-210
(make_beam); a mis-ordered Cint / Float64 would otherwise ship silently."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

SHIM = os.path.join(ROOT, "torj.jl_amd", "julia", "TorJHIP.jl")
HEADER = os.path.join(ROOT, "include", "torj_hip.h")

# Julia ccall type -> the normalised C types it may stand for
JL2C = {
    "Cint": {"int"},
    "Float64": {"double"},
    "Cvoid": {"void"},
    "Cstring": {"char*"},
    "Ptr{Float64}": {"double*"},
    "Ptr{Cint}": {"int*"},
    "Ref{Cint}": {"int*"},
    "Ptr{UInt64}": {"uint64_t*"},
    "Ptr{Cvoid}": {"torj_plasma_t", "void*"},
    "Ptr{Ptr{Cvoid}}": {"torj_plasma_t*"},
    "Ref{TraceCfg}": {"torj_trace_cfg*"},
}


def _split_top(s):
    """Split s at top-level commas (outside (), {}, [])."""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        out.append("".join(cur).strip())
    return out


def _balanced(s, i):
    """Index just past the parenthesis that closes the one at s[i]."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced")


def shim_ccalls():
    src = open(SHIM).read()
    src = re.sub(r"#[^\n]*", "", src)  # comments
    calls = []
    for m in re.finditer(r"ccall\(", src):
        i = m.end() - 1
        body = src[i + 1:_balanced(src, i) - 1]
        parts = _split_top(body)
        sym = re.match(r"\(\s*:(\w+)\s*,\s*libtorj\s*\)", parts[0]).group(1)
        ret = parts[1]
        tys = parts[2].strip()
        assert tys.startswith("(") and tys.endswith(")"), tys
        types = _split_top(tys[1:-1])
        calls.append((sym, ret, types, parts[3:]))
    return calls


def _norm_c(t):
    t = re.sub(r"\bconst\b", "", t)
    t = re.sub(r"\s+", " ", t).strip()
    arr = t.endswith("]")
    t = re.sub(r"\[\d*\]$", "", t).strip()
    stars = t.count("*")
    base = t.replace("*", "").strip()
    if stars == 0 and arr:  # "double x0[3]" (name already removed) -> pointer
        stars = 1
    return base + "*" * stars


def header_prototypes():
    h = open(HEADER).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w \*]*?)\b(torj_\w+)\s*\(([^;{}]*?)\)\s*;", h):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        params = []
        if args.strip() not in ("", "void"):
            for a in _split_top(args):
                a = a.strip()
                arr = re.search(r"\[\d*\]$", a)
                a2 = re.sub(r"\[\d*\]$", "", a).strip()
                a2 = re.sub(r"\b\w+$", "", a2).strip()  # the parameter name
                params.append(_norm_c(a2 + ("[]" if arr else "")))
        protos[name] = (_norm_c(ret), params)
    return protos


def c_struct_fields(name):
    h = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    m = re.search(r"typedef struct \{([^}]*)\}\s*" + name + r"\s*;", h)
    assert m, name
    fields = []
    for decl in m.group(1).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        ty, names = re.match(r"((?:const\s+)?\w+\s*\**)\s*(.*)", decl).groups()
        for nm in names.split(","):
            stars = nm.count("*")
            fields.append((nm.replace("*", "").strip(), _norm_c(ty + "*" * stars)))
    return fields


def test_shim_parses_every_ccall():
    calls = shim_ccalls()
    syms = {c[0] for c in calls}
    # the shim's entry points of the drop-in (make_ray / make_beam path)
    for s in ("torj_abi_version", "torj_plasma_create", "torj_plasma_create_from_coefs",
              "torj_ray_entry_gpu", "torj_trace_beam", "torj_launch_peripheral_rays",
              "torj_shell_volumes", "torj_abs_al_init", "torj_alpha_warm", "torj_beam_comm_info"):
        assert s in syms, s


@pytest.mark.parametrize("call", shim_ccalls(), ids=lambda c: c[0])
def test_ccall_matches_header(call):
    sym, ret, types, actual = call
    protos = header_prototypes()
    assert sym in protos, f"{sym} is not declared in include/torj_hip.h"
    c_ret, c_params = protos[sym]
    assert c_ret in JL2C[ret], f"{sym}: return {ret} vs C {c_ret}"
    assert len(types) == len(c_params), f"{sym}: {len(types)} Julia types vs {len(c_params)} C params"
    assert len(actual) == len(types), f"{sym}: {len(actual)} arguments for {len(types)} types"
    for k, (jt, ct) in enumerate(zip(types, c_params)):
        assert jt in JL2C, f"{sym} arg {k}: unmapped Julia type {jt}"
        assert ct in JL2C[jt], f"{sym} arg {k}: Julia {jt} vs C {ct}"


def test_ccall_symbols_exported():
    L = ctypes.CDLL(os.path.join(ROOT, "torj.jl_amd", "build", "libtorj_hip.so"))
    for sym, *_ in shim_ccalls():
        assert hasattr(L, sym), f"{sym} not exported by libtorj_hip.so"


def test_trace_cfg_field_order_and_types():
    src = re.sub(r"#[^\n]*", "", open(SHIM).read())
    m = re.search(r"struct TraceCfg\s*\n(.*?)\nend", src, flags=re.S)
    jl = re.findall(r"(\w+)::(\w+)", m.group(1))
    c = c_struct_fields("torj_trace_cfg")
    assert [n for n, _ in jl] == [n for n, _ in c]
    for (n, jt), (_, ct) in zip(jl, c):
        assert ct in JL2C[jt], f"TraceCfg.{n}: Julia {jt} vs C {ct}"


def test_abi_versions_agree():
    h = open(HEADER).read()
    v = int(re.search(r"#define TORJ_ABI_VERSION (\d+)", h).group(1))
    jl = int(re.search(r"const ABI_VERSION = (\d+)", open(SHIM).read()).group(1))
    from torj_hip._lib import ABI_VERSION

    assert v == jl == ABI_VERSION


def test_checker_catches_a_swapped_argument(monkeypatch):
    """The check itself: a Cint / Float64 swap in one ccall is reported."""
    calls = shim_ccalls()
    sym, ret, types, actual = next(c for c in calls if c[0] == "torj_trace_beam")
    bad = list(types)
    i = bad.index("Cint")
    bad[i] = "Float64"
    with pytest.raises(AssertionError):
        test_ccall_matches_header((sym, ret, bad, actual))
