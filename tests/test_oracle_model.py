"""CPU oracle model (oracle/model.py) against the reference's own forward() on tiny models
(tests/golden/model_*.npz from make_golden_model.py).  CPU only."""
import numpy as np
import pytest

from model_fixtures import KINDS, load, oracle_grads


# every 336x336 fixture, and two of the SUNRGBD-geometry ones (480x640 LoCa at bs 1; the mixed,
# right-padded [336^2, 480x640] batch through NT-Xent over its 7 real tiles)
@pytest.mark.parametrize("name", list(KINDS) + ["sun_lb", "mix_fb"])
def test_oracle_step_matches_reference(name):
    meta, exp = load(name)
    total, grads = oracle_grads(name)
    assert total == pytest.approx(float(exp["total"]), rel=1e-5)
    names = [str(n) for n in exp["grad_names"]]
    assert sorted(grads) == sorted(names), set(grads) ^ set(names)
    for n, norm, head in zip(names, exp["grad_norms"], exp["grad_heads"]):
        g = grads[n].double()
        assert float(g.norm()) == pytest.approx(float(norm), rel=1e-3, abs=1e-9), n
        np.testing.assert_allclose(g.reshape(-1)[:16].numpy(), head, rtol=2e-3, atol=1e-6 * max(float(norm), 1e-3))
