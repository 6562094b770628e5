"""raftstep — MI355X-native batched Raft step engine (Python host binding).

The engine itself is libraftstep.so (HIP kernels for gfx950 behind the C-ABI
in include/raftstep.h); this package only binds that ABI with ctypes.
"""
from . import abi
from .abi import (CANDIDATE, FOLLOWER, LEADER, STAT_NAMES, default_config, empty_state)
from .engine import Engine, RaftError, load_library, stream_probe, LIB_PATH

__all__ = ["abi", "Engine", "RaftError", "load_library", "stream_probe", "LIB_PATH", "default_config",
           "empty_state", "FOLLOWER", "CANDIDATE", "LEADER", "STAT_NAMES"]
