"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol
include/rr_serdes.h declares; the headers compile as plain C; no GPU compute is called."""
import ctypes
import os
import re
import subprocess

import redrock_old_amd as rr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rr_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = rr.lib()
    syms = declared_symbols("rr_serdes.h")
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/rr_serdes.h but not exported"
    assert sorted(rr.EXPORTS) == syms


def test_library_exports_every_snappy_symbol():
    """include/rr_snappy.h (row f3): every declared function is exported and bound."""
    lib = rr.lib()
    syms = declared_symbols("rr_snappy.h")
    assert len(syms) == 6
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/rr_snappy.h but not exported"
    assert sorted(rr.SNAPPY_EXPORTS) == syms
    assert lib.rr_snappy_max_compressed_length(16384) == 32 + 16384 + 16384 // 6


def test_library_exports_every_rdb_symbol():
    """include/rr_rdb.h (row f4): every declared function is exported."""
    lib = rr.lib()
    syms = declared_symbols("rr_rdb.h")
    assert len(syms) == 5
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/rr_rdb.h but not exported"
    assert sorted(rr.RDB_EXPORTS) == syms


def test_library_exports_every_kv_symbol():
    """include/rr_kv.h (row f2): every declared function is exported."""
    lib = rr.lib()
    syms = declared_symbols("rr_kv.h")
    assert len(syms) == 2
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/rr_kv.h but not exported"
    assert sorted(rr.KV_EXPORTS) == syms


def test_library_exports_every_host_symbol():
    """include/rr_host.h (the host codec behind the compat shim's per-key calls): every declared
    function is exported and bound."""
    lib = rr.lib()
    syms = declared_symbols("rr_host.h")
    assert len(syms) == 7
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/rr_host.h but not exported"
    assert sorted(rr.HOST_EXPORTS) == syms


def test_compat_header_symbols_defined(tmp_path):
    """Every function include/rock_serdes_compat.h declares (the legacy desString / serObject /
    desObject of rock_serdes.h:47-49 and the rr_compat_* batch forms) is defined by the shim,
    redrock_old_amd/compat/rock_serdes_compat.c, compiled as C inside a (model) Redis tree."""
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "rock_serdes_compat.h")).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b([A-Za-z_][A-Za-z_0-9]*)\s*\([^;{]*\)\s*;", txt)))
    assert {"desString", "serObject", "desObject", "rr_compat_des_batch", "rr_compat_ser_batch",
            "rr_compat_rdb_load_batch"} <= set(declared)
    obj = tmp_path / "compat.o"
    subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-DRR_REDIS_TREE", "-c",
                    "-I", os.path.join(ROOT, "tests", "c", "miniredis"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "redrock_old_amd", "compat", "rock_serdes_compat.c"), "-o", str(obj)],
                   check=True)
    nm = subprocess.run(["nm", str(obj)], capture_output=True, text=True, check=True).stdout
    defined = {ln.split()[-1] for ln in nm.splitlines() if " T " in ln}
    for s in declared:
        assert s in defined, f"{s} declared in rock_serdes_compat.h but not defined by the shim"


def test_headers_compile_as_plain_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "rr_serdes.h"\n#include "rr_snappy.h"\n#include "rr_rdb.h"\n#include "rr_kv.h"\n#include "rock_serdes_compat.h"\n'
                   'int main(void){ return (int)sizeof(rr_value) + (int)sizeof(rr_elem) - 32; }\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(tmp_path / "t")], check=True)
    assert subprocess.run([str(tmp_path / "t")]).returncode == 0


def test_struct_layout_matches_numpy():
    assert rr.VALUE_DT.itemsize == 16 and rr.ELEM_DT.itemsize == 16
    assert ctypes.sizeof(rr.Totals) == 32


def test_generator_is_deterministic():
    a = rr.gen_batch(4, 500)
    b = rr.gen_batch(4, 500)
    c = rr.gen_batch(4, 500, seed=123)
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
    assert a[0].shape != c[0].shape or not (a[0] == c[0]).all()


def test_ctx_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    try:
        rr.Engine(0)
    except rr.RRError as e:
        assert "device" in str(e).lower() or "hip" in str(e).lower()
    else:
        raise AssertionError("Engine() must fail without a GPU (no CPU fallback)")
