"""The HIP engine (through the C-ABI) against the same hand-derived KATs that
pin the oracle."""
import pytest

import kat_cases

pytestmark = pytest.mark.gpu


def make_engine(kw):
    from raftstep import Engine
    return Engine(**kw)


@pytest.mark.parametrize("case", kat_cases.ALL, ids=lambda f: f.__name__)
def test_engine_kat(case):
    case(make_engine)
