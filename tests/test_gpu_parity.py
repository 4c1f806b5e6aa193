"""HIP path vs the reference's own outputs on injected physics (golden fixtures) -- needs the MI355X."""
import pytest

from golden_util import SCENARIOS


@pytest.mark.gpu
@pytest.mark.parametrize("name", SCENARIOS)
def test_hip_matches_reference(name):
    from parity_driver import run_parity
    run_parity(name)
