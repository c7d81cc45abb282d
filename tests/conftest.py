import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsng_hip.so)")
    config.addinivalue_line("markers", "oracle_mode(mode): the oracle formulas a test compares against: 'literal' (the "
                                       "reference's text as written) or 'product' (the product's fast-math restatements)")


@pytest.fixture(autouse=True)
def _oracle_mode(request):
    """Every test starts with the oracle mode it states (pytest.mark.oracle_mode, module- or test-level), 'literal'
    when it states none, so no test inherits another's mode (orc_set_literal, oracle/sng_oracle.h)."""
    m = request.node.get_closest_marker("oracle_mode")
    mode = m.args[0] if m else "literal"
    assert mode in ("literal", "product"), mode
    if m is not None or "oracle" in sys.modules:
        import oracle as O
        O.lib().orc_set_literal(1 if mode == "literal" else 0)
        O.lib().orc_set_render_lens(None)   # and no lens left over from another test
        O.lib().orc_set_train_lens(None, 0)
    yield


@pytest.fixture(scope="session")
def synthetic_model():
    from synerfgine_amd import synthetic
    return synthetic.lego_like(seed=1337)


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle as O
    O.lib()
    return O
