"""The committed multigrid histories (tests/golden/mg_history/, made by
tests/golden/make_mg_fixtures.py) that the GPU tests compare against: each
belongs to the density tests/mg_history.py makes, and the cheapest one is
reproduced by the oracle here, so the fixtures cannot drift from the
checker that made them."""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np
import pytest

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import mg_history  # noqa: E402

GOLDEN = HERE / "golden" / "mg_history"


@pytest.mark.parametrize("name", ["parity_128", "parity_256_40", "parity_256_3000", "native_128", "native_256"])
def test_fixture_density(name):
    f = json.loads((GOLDEN / f"{name}.json").read_text())
    rho = mg_history.make_rho(f["size"], f["seed"], f["amp"])
    assert hashlib.sha256(rho.tobytes()).hexdigest() == f["rho_sha256"]
    h = np.array(f["residual"])
    assert len(h) >= 1 and np.all(h > 0)
    if name.startswith("native") or name == "parity_128":
        assert h[-1] <= 1e-10          # converged
    if name == "parity_256_3000":
        assert len(h) == 3000 and 150 < np.argmin(h) < 300 and h[-1] > 1e-3   # the reference algorithm diverges


def test_native_128_fixture_reproduces(built):
    f = json.loads((GOLDEN / "native_128.json").read_text())
    r = mg_history.run("oracle", 128, f["levels"], f["cycle_cap"], f["seed"], f["amp"], native=True)
    assert r["residual"][-1] == f["residual"]
    k = f["phi_stride"]
    assert np.array_equal(r["phi"][::k, ::k, ::k].ravel(), np.array(f["phi_sub"]))
