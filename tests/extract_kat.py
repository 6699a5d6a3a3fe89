"""testExtractEmigrantsXD (test/pusher.test.c:360-545) as a run configuration
and a checker, shared by the oracle test (tests/test_oracle_kat.py) and the
HIP test (tests/test_gpu_reference_kat.py).

The known answers live in tests/golden/reference_outputs.json
("extractEmigrantsXD", made by tests/golden/make_extract_kat.py); this module
only turns them into an ini and compares a run's state with them.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

K = json.loads((Path(__file__).parent / "golden" / "reference_outputs.json").read_text())["kat"]["extractEmigrantsXD"]


def grid_ini_text() -> str:
    """The test's [grid] section (gCreateNeighborhood reads nothing else)."""
    g = {k.split(":")[1]: v for k, v in K["ini"].items() if k.startswith("grid:")}
    return ("[grid]\nnDims=3\nstepSize=1,1,1\nboundaries=PERIODIC,PERIODIC,PERIODIC,PERIODIC,PERIODIC,PERIODIC\n"
            + "".join(f"{k}={v}\n" for k, v in g.items()))


def inputs():
    pos = np.array(K["pos"], dtype=np.float64)
    vel = np.tile(np.array(K["vel"], dtype=np.float64), (len(pos), 1))
    return pos, vel


def check(counts: np.ndarray, records, survivors) -> None:
    """counts: [27, 3] emigrant counts; records(ne) -> [n, 6] emigrants[ne]
    rows (pos, vel) in buffer order; survivors(s) -> (pos, vel) of species
    s's live particles in slot order."""
    exp = np.array(K["expect_nEmigrants"]).reshape(27, 3)
    np.testing.assert_array_equal(counts, exp)
    for ne in range(27):
        if ne == 13:
            continue
        got = records(ne)
        want = np.array(K["expect_emigrants"][str(ne)], dtype=np.float64)
        assert got.shape == want.shape, (ne, got.shape, want.shape)
        np.testing.assert_array_equal(got, want, err_msg=f"emigrants[{ne}]")   # (a copy: exact)
    start = K["iStart"]
    for s, stop in enumerate(K["expect_iStop"]):
        pos, vel = survivors(s)
        assert len(pos) == stop - start[s], (s, len(pos))
        if len(pos) == 0:
            continue
        want = np.zeros((len(pos), 3))
        want[:, 0] = K["expect_survivor_x"]
        want[:, 1:] = K["survivor_yz"]
        np.testing.assert_array_equal(pos, want, err_msg=f"survivors of species {s}")
        np.testing.assert_array_equal(vel, np.tile(K["vel"], (len(pos), 1)))
