"""CPU: the checkpoint file format's reader/writer (raftstep.checkpoint) —
version 1 (no iso_victim) and 2 round trips, CRC32C trailer rejection, and
the vectorised CRC32C against the standard check value and the oracle's
bytewise implementation (oracle_crc32c)."""
import numpy as np
import pytest

import oracle
from raftstep import abi, checkpoint


def random_view(rng, G=37, R=5, K=8):
    st = abi.empty_state(G, R, K)
    for k, a in st.items():
        st[k] = rng.integers(0, 100, a.shape).astype(a.dtype)
    return st


@pytest.mark.parametrize("version", [1, 2])
def test_write_read_round_trip(tmp_path, version):
    rng = np.random.default_rng(version)
    cfg = abi.default_config(replicas=5, groups=37, ring_depth=8, seed=0xABC)
    st = random_view(rng)
    p = tmp_path / "ck.bin"
    checkpoint.write(p, cfg, st, version=version)
    cfg2, st2 = checkpoint.read(p)
    assert bytes(cfg2) == bytes(cfg)
    for k in abi.STATE_FIELDS:
        if version == 1 and k == "iso_victim":
            assert k not in st2
            continue
        assert np.array_equal(st2[k], st[k]), k
    data = bytearray(p.read_bytes())
    data[200] ^= 1
    p.write_bytes(bytes(data))
    with pytest.raises(ValueError, match="CRC32C"):
        checkpoint.read(p)
    checkpoint.read(p, verify=False)   # (structure only)


def test_crc32c_vectorised_matches_bytewise():
    assert checkpoint.crc32c(b"123456789") == 0xE3069283   # RFC 3720 check value
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 8, 4095, 8192 * 2 + 5, (1 << 17) + 3, 3 << 20):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert checkpoint.crc32c(d) == oracle.crc32c(d), n
