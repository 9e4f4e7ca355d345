"""CPU pin of the LuaJIT binding (lua/multigrid-poisson/hip.lua) to the C ABI (include/mgpoisson.h).

No Lua runtime exists in this image, so hip.lua cannot run here.  Its ``ffi.cdef[[...]]`` block is
C, though: it is compiled with gcc in ONE translation unit after the real header, so any function
prototype or typedef that drifts from the header is a "conflicting types" error.  The cdef's own
copy of ``struct mgp_opts`` (a struct cannot be defined twice in C) is renamed and pinned field by
field with ``_Static_assert`` on offsetof / sizeof against the header's.  The ctypes mirror
(mgpoisson/_lib.py) is checked against the same offsets, compiled and printed by gcc.
"""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER_DIR = os.path.join(ROOT, "include")
LUA = os.path.join(ROOT, "lua-multigrid-poisson_amd", "lua", "multigrid-poisson", "hip.lua")


def _cdef():
    text = open(LUA).read()
    m = re.search(r"ffi\.cdef\s*\[\[(.*?)\]\]", text, flags=re.S)
    assert m, "hip.lua has no ffi.cdef[[...]] block"
    return m.group(1)


def _split_struct(cdef):
    """(cdef without its mgp_opts definition, [(type, name, array) fields of that definition])."""
    m = re.search(r"typedef\s+struct\s+mgp_opts\s*\{(.*?)\}\s*mgp_opts\s*;", cdef, flags=re.S)
    assert m, "hip.lua's cdef must define mgp_opts"
    fields = []
    for decl in m.group(1).split(";"):
        decl = re.sub(r"/\*.*?\*/", "", decl).strip()
        if not decl:
            continue
        typ, rest = decl.rsplit(None, 1) if "," not in decl else (decl.split()[0], decl[len(decl.split()[0]):])
        for name in rest.split(","):
            name = name.strip()
            arr = re.match(r"(\w+)\s*\[(\d+)\]", name)
            fields.append((typ, arr.group(1) if arr else name, int(arr.group(2)) if arr else 0))
    return cdef[:m.start()] + cdef[m.end():], fields


def _gcc(src, tmp_path, run=False):
    c = tmp_path / "t.c"
    c.write_text(src)
    exe = tmp_path / "t"
    cmd = ["gcc", "-std=c11", "-Wall", "-Werror", f"-I{HEADER_DIR}", str(c)] + (["-o", str(exe)] if run else ["-fsyntax-only"])
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    if run:
        return subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    return ""


def test_cdef_prototypes_agree_with_header(tmp_path):
    rest, fields = _split_struct(_cdef())
    lua_struct = "typedef struct lua_mgp_opts {\n" + "".join(
        f"    {t} {n}{'[%d]' % a if a else ''};\n" for t, n, a in fields) + "} lua_mgp_opts;\n"
    asserts = [f'_Static_assert(sizeof(lua_mgp_opts) == sizeof(mgp_opts), "sizeof mgp_opts");']
    for t, n, a in fields:
        asserts.append(f'_Static_assert(offsetof(lua_mgp_opts, {n}) == offsetof(mgp_opts, {n}), "offset {n}");')
        asserts.append(f'_Static_assert(sizeof(((lua_mgp_opts*)0)->{n}) == sizeof(((mgp_opts*)0)->{n}), "size {n}");')
    src = ("#include <stddef.h>\n#include <stdint.h>\n#include \"mgpoisson.h\"\n" + rest + "\n" + lua_struct
           + "\n".join(asserts) + "\n")
    _gcc(src, tmp_path)


def test_cdef_declares_only_header_functions_and_the_ones_it_calls():
    cdef = _cdef()
    hdr = open(os.path.join(HEADER_DIR, "mgpoisson.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = set(re.findall(r"\b(mgp_[a-z_0-9]+)\s*\(", cdef))
    in_header = set(re.findall(r"\b(mgp_[a-z_0-9]+)\s*\(", hdr))
    assert declared <= in_header, declared - in_header
    used = set(re.findall(r"lib\.(mgp_[a-z_0-9]+)", open(LUA).read()))
    assert used <= declared, used - declared


def test_header_asserts_opts_size(tmp_path):
    """The header pins sizeof(mgp_opts) itself; a changed struct fails every C/C++ consumer's build."""
    out = _gcc('#include <stdio.h>\n#include <stddef.h>\n#include "mgpoisson.h"\nint main(void){printf("%zu\\n", '
               'sizeof(mgp_opts));return 0;}\n', tmp_path, run=True)
    assert int(out) == 232
    assert "_Static_assert(sizeof(mgp_opts) == 232" in open(os.path.join(HEADER_DIR, "mgpoisson.h")).read()


def test_ctypes_mirror_offsets(tmp_path):
    from mgpoisson import _lib

    names = [f[0] for f in _lib.MGPOpts._fields_]
    prog = "#include <stdio.h>\n#include <stddef.h>\n#include \"mgpoisson.h\"\nint main(void){\n" + "".join(
        f'printf("{n} %zu\\n", offsetof(mgp_opts, {n}));\n' for n in names) + "return 0;}\n"
    out = _gcc(prog, tmp_path, run=True)
    c_off = {l.split()[0]: int(l.split()[1]) for l in out.splitlines()}
    for n in names:
        assert getattr(_lib.MGPOpts, n).offset == c_off[n], n


@pytest.mark.parametrize("name", ["mgp_group_create", "mgp_group_cycles", "mgp_residual_norm", "mgp_get_planes"])
def test_cdef_binds_round2_entry_points(name):
    """The Lua host reaches the single-process multi-GPU group and the new reductions / plane I/O."""
    assert re.search(rf"\b{name}\s*\(", _cdef()), name
