"""Static checks of the Julia drop-in shim against the C-ABI (no Julia in the image).

The shim (sharedmemsparselu.jl_amd/julia/src/SharedMemSparseLU.jl) is the reference-side binding
of `ParallelSparseLU(A)` / `lu!` / `ldiv!` (/root/reference/src/SharedMemSparseLU.jl:64, :245,
:286).  Without a Julia interpreter it can only break silently, as it did when `smlu_opts` gained
a field and `default_opts()` kept passing one value too few.  These tests parse both sides:

* `SmluOpts` has the fields of `smlu_opts` (include/smlu.h) in order, with matching types;
* the positional `SmluOpts(...)` call in `default_opts()` passes one value per field;
* every `:smlu_*` symbol the shim `ccall`s is declared in the header, and the ccall's argument
  type tuple has the header's parameter count (for every symbol a conditional ccall may pick);
* `p`/`q` come back as `Vector{Ti}` (the reference's `p::Vector{Ti}`, :49-50);
* the copy in INTEGRATION.md is the file verbatim and names only symbols the header declares.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "sharedmemsparselu.jl_amd", "julia", "src", "SharedMemSparseLU.jl")
HEADER = os.path.join(ROOT, "include", "smlu.h")

C2JL = {"int64_t": "Int64", "int32_t": "Int32", "double": "Float64"}


def _header():
    src = open(HEADER).read()
    return re.sub(r"/\*.*?\*/", "", src, flags=re.S)


def header_opts_fields():
    body = re.search(r"typedef struct smlu_opts \{(.*?)\} smlu_opts;", _header(), flags=re.S).group(1)
    fields = []
    for m in re.finditer(r"(\w+)\s+(\w+)(\[(\d+)\])?\s*;", body):
        ctype, name, _, dim = m.groups()
        jt = C2JL[ctype]
        fields.append((name, f"NTuple{{{dim},{jt}}}" if dim else jt))
    return fields


def header_prototypes():
    """name -> parameter count of every smlu_* function declared in the header."""
    out = {}
    for m in re.finditer(r"\b(smlu_\w+)\s*\(([^;{]*?)\)\s*;", _header(), flags=re.S):
        name, params = m.group(1), m.group(2).strip()
        if params in ("", "void"):
            out[name] = 0
        else:
            out[name] = len(_split_top(params))
    return out


def _split_top(s):
    """Split at commas outside (), {}, []."""
    parts, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return [p.strip() for p in parts if p.strip()]


def _balanced(s, i):
    """s[i] == '(' -> index just past its matching ')'."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return j + 1
    raise AssertionError("unbalanced parentheses")


def _strip_comments(src):
    return "\n".join(re.sub(r"#.*$", "", ln) for ln in src.splitlines())


def shim_ccalls(src):
    """(symbols, n_arg_types) for every ccall in the shim."""
    src = _strip_comments(src)
    calls = []
    for m in re.finditer(r"\bccall\(", src):
        end = _balanced(src, m.end() - 1)
        args = _split_top(src[m.end():end - 1])
        target, types = args[0], args[2]
        syms = re.findall(r":(smlu_\w+)", target)
        assert syms, f"ccall without a smlu_ symbol: {target}"
        assert types.startswith("(") and types.endswith(")"), f"argument types not a tuple: {types}"
        calls.append((syms, len(_split_top(types[1:-1]))))
    return calls


def test_opts_struct_matches_header():
    src = open(SHIM).read()
    body = re.search(r"mutable struct SmluOpts\s*(.*?)\n\s*end", src, flags=re.S).group(1)
    jl = [(n, t.replace(" ", "")) for n, t in re.findall(r"(\w+)::([\w{},\s]+?)(?:;|\n|$)", body)]
    assert jl == header_opts_fields()


def test_default_opts_arity():
    src = open(SHIM).read()
    call = re.search(r"SmluOpts\((.*?)\)\n", src).group(1)
    assert len(_split_top(call)) == len(header_opts_fields())


def test_ccalls_match_prototypes():
    protos = header_prototypes()
    calls = shim_ccalls(open(SHIM).read())
    assert len(calls) >= 15
    for syms, nargs in calls:
        for s in syms:
            assert s in protos, f"shim calls {s}, not declared in include/smlu.h"
            assert protos[s] == nargs, f"{s}: shim passes {nargs} argument types, header has {protos[s]}"


def test_constructors_and_entry_points_present():
    calls = {s for syms, _ in shim_ccalls(open(SHIM).read()) for s in syms}
    for s in ("smlu_create", "smlu_create_i32", "smlu_create_z", "smlu_create_with_pivots",
              "smlu_refactor", "smlu_refactor_csc", "smlu_solve", "smlu_solve_multi",
              "smlu_lsolve", "smlu_rsolve", "smlu_get_factors", "smlu_destroy",
              "smlu_rccl_unique_id", "smlu_dist_create_rccl"):
        assert s in calls, s


def test_permutations_come_back_as_Ti():
    src = open(SHIM).read()
    assert "s === :p && return Vector{Ti}(p)" in src
    assert "s === :q && return Vector{Ti}(q)" in src


def test_integration_copy_is_verbatim_and_current():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"```julia\n(# Julia ccall shim.*?\nend\n)```", doc, flags=re.S)
    assert m and m.group(1) == open(SHIM).read(), "INTEGRATION.md's shim copy is stale"
    protos = header_prototypes()
    for s in set(re.findall(r"\b(smlu_\w+)\b", doc)):
        assert s in protos or s in ("smlu_opts", "smlu_transport", "smlu_handle", "smlu_plan"), \
            f"INTEGRATION.md names {s}, which include/smlu.h does not declare"
