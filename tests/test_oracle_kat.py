"""The oracle (CPU restatement of main.go) against the hand-derived KATs of
SURVEY.md Appendix B — this is what pins the oracle (no Go toolchain exists
here and the reference ships no tests or golden vectors)."""
import pytest

import kat_cases


def make_oracle(kw):
    import oracle
    return oracle.Oracle(**kw)


@pytest.mark.parametrize("case", kat_cases.ALL, ids=lambda f: f.__name__)
def test_oracle_kat(case, oracle_mod):
    case(make_oracle)
