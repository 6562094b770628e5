"""CPU-side checks of the C-ABI boundary: the library loads and exports every
function include/raftstep.h declares; record layouts match the header. No
compute calls (there is no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
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


@pytest.mark.parametrize("field,value,msg", [
    ("groups", (1 << 30) // 3 + 1, "too many groups"),   # Gp*R*4 would wrap the 32-bit byte offsets
    ("groups", 0, "groups must be"),
    ("replicas", 9, "replicas"),
    ("ring_depth", 24, "power of two"),
    ("isolate_leader", 2, "isolate_leader"),
    ("ticks_per_launch", 65, "ticks_per_launch"),
    ("debug_flags", 2, "debug_flags"),
])
def test_engine_create_rejects_bad_configs_before_touching_a_gpu(field, value, msg):
    """Config validation runs before any HIP call, so it is checkable here."""
    lib = engine.load_library()
    c = abi.default_config(**{field: value})
    h = C.c_void_p()
    rc = lib.raft_engine_create(C.byref(c), C.byref(h))
    assert rc == abi.RAFT_EINVAL and not h.value
    assert msg in lib.raft_last_error().decode()


NPL = 9   # int32 rows per group record (raft_device.hpp), padded to 16 B: groups * recw * 4 < 2^32


def test_largest_engine_size_is_accepted_by_validation():
    """The largest group count whose records keep 32-bit byte offsets passes the
    size checks (then fails only for lack of a device here); one more block of
    256 groups is refused."""
    lib = engine.load_library()
    for R in (1, 5, 7):
        recw = (NPL * R + 3) & ~3
        top = ((1 << 32) - 1) // (recw * 4) // 256 * 256
        c = abi.default_config(replicas=R, groups=top)
        h = C.c_void_p()
        rc = lib.raft_engine_create(C.byref(c), C.byref(h))
        assert rc != abi.RAFT_EINVAL or "too many groups" not in lib.raft_last_error().decode()
        c = abi.default_config(replicas=R, groups=top + 1)
        rc = lib.raft_engine_create(C.byref(c), C.byref(h))
        assert rc == abi.RAFT_EINVAL and "too many groups" in lib.raft_last_error().decode()


def test_coerce_state_checks_dtype_shape_and_optional_fields():
    G, R, K = 3, 5, 8
    st = abi.empty_state(G, R, K)
    st["term"] = st["term"].astype(np.int64) + 7          # int64 after numpy arithmetic: converted, not misread
    out = abi.coerce_state(st, G, R, K)
    assert out["term"].dtype == np.int32 and (out["term"] == 7).all()
    for k in abi.OPTIONAL_ON_LOAD:                          # optional fields may be absent
        del st[k]
    out = abi.coerce_state(st, G, R, K)
    assert not set(abi.OPTIONAL_ON_LOAD) & set(out)
    bad = dict(st, last=np.zeros((G, R - 1), np.int32))     # short array: refused, never read past its end
    with pytest.raises(ValueError, match="shape"):
        abi.coerce_state(bad, G, R, K)
    bad = dict(st, term=np.full((G, R), 1 << 40))           # does not fit int32
    with pytest.raises(ValueError, match="fit"):
        abi.coerce_state(bad, G, R, K)
    bad = dict(st, commit=np.zeros((G, R), np.float32))
    with pytest.raises(TypeError):
        abi.coerce_state(bad, G, R, K)
    missing = {k: v for k, v in st.items() if k != "fault"}
    with pytest.raises(KeyError):
        abi.coerce_state(missing, G, R, K)


def test_results_altering_env_knob_is_refused_without_the_debug_flag(monkeypatch):
    """RAFTSTEP_DIAG_LEAN skips work (timing diagnostics): raft_engine_create
    refuses it unless debug_flags says wrong results are acceptable. The check
    runs before any HIP call."""
    lib = engine.load_library()
    h = C.c_void_p()
    monkeypatch.setenv("RAFTSTEP_DIAG_LEAN", "64")
    c = abi.default_config(groups=256)
    assert lib.raft_engine_create(C.byref(c), C.byref(h)) == abi.RAFT_EINVAL and not h.value
    assert "RAFTSTEP_DIAG_LEAN" in lib.raft_last_error().decode()
    c = abi.default_config(groups=256, debug_flags=abi.DEBUG_ALLOW_WRONG_RESULTS)
    rc = lib.raft_engine_create(C.byref(c), C.byref(h))   # accepted by validation (no device here)
    assert rc != abi.RAFT_EINVAL or "RAFTSTEP_DIAG_LEAN" not in lib.raft_last_error().decode()
    if h.value:
        lib.raft_engine_destroy(h)


def test_reserved_config_words_must_be_zero():
    lib = engine.load_library()
    c = abi.default_config()
    c.reserved[1] = 7
    h = C.c_void_p()
    assert lib.raft_engine_create(C.byref(c), C.byref(h)) == abi.RAFT_EINVAL
    assert "reserved" in lib.raft_last_error().decode()
