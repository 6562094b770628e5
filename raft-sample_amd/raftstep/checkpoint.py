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


def read(path):
    """(raft_config, {field: array}) of a checkpoint; shapes as abi.state_shapes."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != MAGIC:
        raise ValueError(f"{path}: not a raftstep checkpoint")
    version, nfields = np.frombuffer(data, "<u4", 2, 8)
    if version != VERSION:
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
    want = int(np.frombuffer(data, "<u4", 1, off)[0])
    got = crc32c(data[:off])
    if got != want:
        raise ValueError(f"{path}: CRC32C mismatch (file {want:08x}, computed {got:08x})")
    return cfg, st


def _crc32c_table():
    t = np.zeros(256, np.uint32)
    for b in range(256):
        c = b
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 & -(c & 1))
        t[b] = c
    return [int(x) for x in t]


_TAB = None


def crc32c(data):
    """CRC32C (Castagnoli) of a byte string, the checkpoint trailer's definition.
    Slice-by-8 over 8-byte words in numpy, bytewise tail."""
    global _TAB
    if _TAB is None:
        base = np.array(_crc32c_table(), np.uint32)
        tabs = [base]
        for _ in range(7):
            prev = tabs[-1]
            tabs.append((prev >> np.uint32(8)) ^ base[prev & np.uint32(255)])
        _TAB = tabs
    T = _TAB
    b = np.frombuffer(bytes(data), np.uint8)
    c = 0xFFFFFFFF
    n8 = len(b) // 8
    if n8:
        w = b[:n8 * 8].reshape(n8, 8)
        lo = (w[:, 0].astype(np.uint32) | (w[:, 1].astype(np.uint32) << 8) |
              (w[:, 2].astype(np.uint32) << 16) | (w[:, 3].astype(np.uint32) << 24))
        hi = w[:, 4:8]
        lo_l, hi_l = lo.tolist(), hi.tolist()
        t0, t1, t2, t3, t4, t5, t6, t7 = (x.tolist() for x in T)
        for i in range(n8):
            x = c ^ lo_l[i]
            h = hi_l[i]
            c = (t7[x & 255] ^ t6[(x >> 8) & 255] ^ t5[(x >> 16) & 255] ^ t4[x >> 24] ^
                 t3[h[0]] ^ t2[h[1]] ^ t1[h[2]] ^ t0[h[3]])
    t0 = T[0].tolist()
    for x in b[n8 * 8:].tolist():
        c = (c >> 8) ^ t0[(c ^ x) & 255]
    return c ^ 0xFFFFFFFF
