"""CPU-side checks of the C-ABI boundary: the library loads and exports every
function include/raftstep.h declares; record layouts match the header. No
compute calls (there is no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from raftstep import abi, engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "raftstep.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(raft_[a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_header_declares_the_expected_surface():
    fns = declared_functions()
    assert set(fns) == set(abi.SIGNATURES), set(fns) ^ set(abi.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = engine.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}$", out, flags=re.M), name


def test_record_layouts_match_header(tmp_path):
    prog = tmp_path / "sz.c"
    prog.write_text('#include <stdio.h>\n#include "%s"\nint main(void){printf("%%zu %%zu %%zu %%zu %%zu %%zu '
                    '%%zu %%zu %%zu %%zu\\n", sizeof(raft_config), sizeof(raft_ae_req), sizeof(raft_ae_resp), '
                    'sizeof(raft_log_entry), sizeof(raft_vote_req), sizeof(raft_vote_resp), sizeof(raft_group_op), '
                    'sizeof(raft_op_result), sizeof(raft_state_view), sizeof(raft_tick_stats));return 0;}\n' % HEADER)
    exe = tmp_path / "sz"
    subprocess.run(["gcc", str(prog), "-o", str(exe)], check=True)
    sizes = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    assert sizes == [C.sizeof(abi.Config), abi.AE_REQ.itemsize, abi.AE_RESP.itemsize, abi.LOG_ENTRY.itemsize,
                     abi.VOTE_REQ.itemsize, abi.VOTE_RESP.itemsize, abi.GROUP_OP.itemsize, abi.OP_RESULT.itemsize,
                     C.sizeof(abi.StateView), C.sizeof(abi.TickStats)]


def test_config_default_matches_python_defaults():
    lib = engine.load_library()
    c = abi.Config()
    lib.raft_config_default(C.byref(c))
    py = abi.default_config()
    for name, _ in abi.Config._fields_:
        if name == "reserved":
            continue
        assert getattr(c, name) == getattr(py, name), name


def test_library_has_no_cpu_path():
    """The product library must not contain or link the oracle."""
    out = subprocess.run(["nm", "-D", engine.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in out
    deps = subprocess.run(["ldd", engine.LIB_PATH], capture_output=True, text=True).stdout
    assert "liboracle" not in deps


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(engine.RaftError):
        engine.load_library(str(tmp_path / "nope.so"))
    engine._lib = None
    engine.load_library()
