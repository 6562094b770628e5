"""GPU: the HIP engine reproduces the committed golden traces bit for bit."""
import pytest

import golden_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", golden_check.NAMES)
def test_engine_matches_golden(name):
    from raftstep import Engine
    golden_check.check(lambda kw: Engine(**kw), name)
