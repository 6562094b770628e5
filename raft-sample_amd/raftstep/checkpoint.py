"""Reader of raft_checkpoint_save files.

The file is written and verified (CRC32C trailer) by the C-ABI
(raft_checkpoint_save / raft_checkpoint_load in engine.cpp); this reader only
parses it into (config, canonical state dict) so that a checkpoint can be
inspected with numpy or loaded into another implementation of the surface
(e.g. the CPU oracle in tests).

Layout (little endian):
  header  : magic "RAFTCKPT" | u32 version | u32 nfields | raft_config (120 B)
  fields  : nfields x { char name[12] | u32 elem | u64 count | count*elem bytes }
  trailer : u32 CRC32C of everything before it
"""
import ctypes as C

import numpy as np

from . import abi

MAGIC = b"RAFTCKPT"
VERSION = 1
_DTYPES = {"role": np.uint8, "voted": np.uint8, "fault": np.uint8, "log_value": np.int64, "log_crc": np.uint32}


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
    return cfg, st
