"""Reader of raft_checkpoint_save files.

The file is written and verified (CRC32C trailer) by the C-ABI
(raft_checkpoint_save / raft_checkpoint_load in engine.cpp); this reader only
parses it into (config, canonical state dict) so that a checkpoint can be
inspected with numpy or loaded into another implementation of the surface
(e.g. the CPU oracle in tests); it verifies the CRC32C trailer first.

Layout (little endian):
  header  : magic "RAFTCKPT" | u32 version | u32 nfields | raft_config (120 B)
  fields  : nfields x { char name[12] | u32 elem | u64 count | count*elem bytes }
  trailer : u32 CRC32C of everything before it
"""
import ctypes as C

import numpy as np

from . import abi

MAGIC = b"RAFTCKPT"
VERSION = 2
_DTYPES = {"role": np.uint8, "voted": np.uint8, "fault": np.uint8, "log_value": np.int64, "log_crc": np.uint32,
           "iso_victim": np.uint8}


def read(path, verify=True):
    """(raft_config, {field: array}) of a checkpoint; shapes as abi.state_shapes.
    Version 1 files (before leader isolation) have no iso_victim field. The
    CRC32C trailer is verified unless verify=False."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != MAGIC:
        raise ValueError(f"{path}: not a raftstep checkpoint")
    version, nfields = np.frombuffer(data, "<u4", 2, 8)
    if version not in (1, VERSION):
        raise ValueError(f"{path}: checkpoint version {version} unsupported")
    cfg = abi.Config.from_buffer_copy(data[16:16 + C.sizeof(abi.Config)])
    shapes = abi.state_shapes(cfg.groups, cfg.replicas, cfg.ring_depth)
    off = 16 + C.sizeof(abi.Config)
    st = {}
    for _ in range(int(nfields)):
        name = data[off:off + 12].rstrip(b"\0").decode()
        elem = int(np.frombuffer(data, "<u4", 1, off + 12)[0])
        count = int(np.frombuffer(data, "<u8", 1, off + 16)[0])
        off += 24
        shape, dt = shapes[name]
        dt = np.dtype(_DTYPES.get(name, dt))
        if dt.itemsize != elem or count != int(np.prod(shape)):
            raise ValueError(f"{path}: field {name} has {count} x {elem} B")
        st[name] = np.frombuffer(data, dt, count, off).reshape(shape).copy()
        off += count * elem
    if off + 4 != len(data):
        raise ValueError(f"{path}: {len(data) - off} trailing bytes, expected the 4-byte CRC32C")
    if verify:
        want = int(np.frombuffer(data, "<u4", 1, off)[0])
        got = crc32c(memoryview(data)[:off])
        if got != want:
            raise ValueError(f"{path}: CRC32C mismatch (file {want:08x}, computed {got:08x})")
    return cfg, st


def write(path, cfg, state, version=VERSION):
    """Writes (cfg, canonical state) in the raft_checkpoint_save format (version
    1 omits iso_victim); raft_checkpoint_load / read() accept it."""
    shapes = abi.state_shapes(cfg.groups, cfg.replicas, cfg.ring_depth)
    names = list(abi.STATE_FIELDS) if version >= 2 else [k for k in abi.STATE_FIELDS if k != "iso_victim"]
    out = bytearray(MAGIC)
    out += np.array([version, len(names)], "<u4").tobytes()
    out += bytes(cfg)
    for name in names:
        shape, dt = shapes[name]
        dt = np.dtype(_DTYPES.get(name, dt))
        a = np.zeros(shape, dt) if state.get(name) is None else np.ascontiguousarray(state[name], dt)
        out += name.encode().ljust(12, b"\0")
        out += np.array([dt.itemsize], "<u4").tobytes() + np.array([a.size], "<u8").tobytes()
        out += a.tobytes()
    out += np.array([crc32c(bytes(out))], "<u4").tobytes()
    with open(path, "wb") as f:
        f.write(bytes(out))


_TAB = None


def _tables():
    """Slice-by-8 CRC32C (Castagnoli, reflected 0x82F63B78) tables T[0..7]."""
    global _TAB
    if _TAB is None:
        base = np.zeros(256, np.uint32)
        for b in range(256):
            c = b
            for _ in range(8):
                c = (c >> 1) ^ (0x82F63B78 & -(c & 1))
            base[b] = c
        tabs = [base]
        for _ in range(7):
            prev = tabs[-1]
            tabs.append((prev >> np.uint32(8)) ^ base[prev & np.uint32(255)])
        _TAB = tabs
    return _TAB


def _serial(c, b):
    """Register update over bytes b from register c (no pre/post inversion)."""
    t0 = _tables()[0].tolist()
    for x in b.tolist():
        c = (c >> 8) ^ t0[(c ^ x) & 255]
    return c


def _zeros_op(nbytes):
    """The register map of nbytes zero bytes (linear over GF(2)) as the images
    of the 32 unit registers, by repeated squaring."""
    t0 = _tables()[0].tolist()
    one = [((1 << k) >> 8) ^ t0[(1 << k) & 255] for k in range(32)]   # one zero byte

    def apply(op, x):
        y = 0
        k = 0
        while x:
            if x & 1:
                y ^= op[k]
            x >>= 1
            k += 1
        return y

    res = [1 << k for k in range(32)]
    sq = one
    while nbytes:
        if nbytes & 1:
            res = [apply(sq, v) for v in res]
        sq = [apply(sq, v) for v in sq]
        nbytes >>= 1
    return res


def crc32c(data):
    """CRC32C (Castagnoli) of a byte string, the checkpoint trailer's
    definition. The register update is linear over GF(2): reg(s, A||B) =
    Z_|B|(reg(s, A)) ^ reg(0, B). The data is cut into 64-KiB chunks whose
    registers (from 0) are computed side by side with numpy slice-by-8, then
    chained through the 32x32 map Z of one chunk of zeros; the tail is
    bytewise. Chunks of 4 KiB .. 1 MiB, about 32K of them: a multi-GB
    checkpoint verifies in seconds."""
    b = np.frombuffer(data, np.uint8)
    T = _tables()
    n = len(b)
    _CHUNK = 4096
    while _CHUNK < (1 << 20) and n // _CHUNK > 32768:
        _CHUNK *= 2
    nch = n // _CHUNK
    c = 0xFFFFFFFF
    if nch >= 2:
        w = b[:nch * _CHUNK].reshape(nch, _CHUNK // 8, 8)
        # word j of every chunk contiguous (one row per step)
        lo = np.ascontiguousarray(np.ascontiguousarray(w[:, :, :4]).view("<u4")[:, :, 0].T)
        hi = np.ascontiguousarray(np.ascontiguousarray(w[:, :, 4:]).view("<u4")[:, :, 0].T)
        r = np.zeros(nch, np.uint32)
        m = np.uint32(255)
        for j in range(_CHUNK // 8):
            x = r ^ lo[j]
            h = hi[j]
            r = (T[7][x & m] ^ T[6][(x >> 8) & m] ^ T[5][(x >> 16) & m] ^ T[4][x >> 24] ^
                 T[3][h & m] ^ T[2][(h >> 8) & m] ^ T[1][(h >> 16) & m] ^ T[0][h >> 24])
        op = _zeros_op(_CHUNK)
        zt = [[0] * 256 for _ in range(4)]   # the map as four byte tables
        for q in range(4):
            for v in range(256):
                y = 0
                for k in range(8):
                    if (v >> k) & 1:
                        y ^= op[8 * q + k]
                zt[q][v] = y
        z0, z1, z2, z3 = zt
        for ri in r.tolist():
            c = z0[c & 255] ^ z1[(c >> 8) & 255] ^ z2[(c >> 16) & 255] ^ z3[c >> 24] ^ ri
        c = _serial(c, b[nch * _CHUNK:])
    else:
        c = _serial(c, b)
    return c ^ 0xFFFFFFFF
