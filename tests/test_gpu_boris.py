"""Boris pusher extension on the MI355X path (methods:acc = puBoris3D1KE,
pinc_hip_boris) against the oracle restatement (tests/test_oracle_boris.py
pins the restatement by the rotation's invariants; the reference's own
puBoris3D1 rotates the wrong particle and is never called, so there is no
reference output: parity unpinned against the reference, pinned against the
algorithm).  Same initial state on both sides; the deposit's atomics reorder
sums, so fields and through them particles agree to rounding."""
import numpy as np
import pytest

import orc
from pinc_amd import configs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sim_cls(built):
    from pinc_amd import Sim
    return Sim


@pytest.mark.parametrize("name,kw,bext,fused", [
    ("cold3d", {}, "0,0,1e-4", "1"),
    ("warm", {"true_size": (32, 32, 32), "ppc": 8, "nalloc_pc": 16, "levels": 3}, "1e-4,-2e-4,3e-4", "1"),
    ("warm", {"true_size": (32, 32, 32), "ppc": 8, "nalloc_pc": 16, "levels": 3}, "1e-4,-2e-4,3e-4", "0"),
])
def test_boris_matches_oracle(sim_cls, name, kw, bext, fused):
    cfg = configs.config(name, **kw)
    cfg["methods"]["acc"] = "puBoris3D1KE"
    cfg["fields"]["BExt"] = bext
    cfg["population"]["fused"] = fused
    ini = configs.write_ini(cfg)
    maxwell = name == "warm"
    w = orc.World(ini)
    w.init(perturb=not maxwell, maxwell=maxwell, seed=11)
    w.init_fields()
    with sim_cls(ini, maxwell=maxwell, perturb=not maxwell, seed=11) as s:
        s.init()
        for sp in range(2):
            vo = w.particles(sp)[1]
            vg = s.particles(sp)[1]
            np.testing.assert_allclose(vg, vo, rtol=0, atol=1e-12 * np.abs(vo).max())
        for n in range(4):
            s.step()
            w.step()
            ke, pe, _ = s.energy()
            ke_o, pe_o = w.energy()
            assert abs(ke - ke_o) <= 1e-9 * abs(ke_o), (n, ke, ke_o)
            assert abs(pe - pe_o) <= 1e-8 * abs(pe_o) + 1e-12, (n, pe, pe_o)
            for sp in range(2):
                assert s.count(sp) == w.count(sp)


def test_boris_rejects_non_3d(built):
    """puSanity (pusher.c:1047, as puBoris3D1_set calls it): a 2-D
    run with the 3-D Boris pusher stops with msg(ERROR), which exits the
    process (io.c:214-215), so it runs in a child process."""
    import subprocess
    import sys
    cfg = configs.config("langmuir2d")
    cfg["methods"]["acc"] = "puBoris3D1KE"
    ini = configs.write_ini(cfg)
    code = f"from pinc_amd import Sim\nwith Sim({str(ini)!r}) as s:\n    s.init()\n"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       cwd=str(configs.__file__).rsplit("/pinc_amd/", 1)[0])
    assert r.returncode != 0
    assert "puBoris3D1KE" in r.stderr and "nDims=3" in r.stderr, r.stderr[-2000:]
