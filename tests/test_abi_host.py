"""C-ABI and host-logic checks that need no GPU.

* Both native libraries load and export every function their header
  declares (include/pinc_hip.h -> libpinc_hip.so, include/pinc.h ->
  libpinc.so).  No compute calls are made.
* Pure host logic of the product library (ini parsing, units
  normalisation, neighbour maps) agrees with the reference's known answers
  and with the oracle.
"""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLD = json.loads((ROOT / "tests" / "golden" / "reference_outputs.json").read_text())["kat"]


@pytest.fixture(scope="module")
def lib(built):
    from pinc_amd import _lib
    return _lib


@pytest.mark.parametrize("header,which", [("pinc_hip.h", "HIP"), ("pinc.h", "HOST")])
def test_header_symbols_exported(lib, header, which):
    names = lib.header_symbols(ROOT / "include" / header)
    assert len(names) > 20
    so = getattr(lib, which)
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, f"{header}: not exported: {missing}"


def test_product_has_no_oracle_dependency():
    """The product libraries and package never reference the oracle."""
    for p in list((ROOT / "pinc_amd").rglob("*.py")) + list((ROOT / "pinc_amd").rglob("*.c")) + \
            list((ROOT / "pinc_amd").rglob("*.hip")):
        text = p.read_text()
        assert "import orc" not in text and "liborc" not in text and "orc_" not in text, p


class MpiInfo(C.Structure):
    """include/pinc.h's MpiInfo: core.h:112-138's fields in core.h's order,
    the RCCL communicator appended."""
    _fields_ = [("mpiRank", C.c_int), ("mpiSize", C.c_int), ("nDims", C.c_int),
                ("subdomain", C.POINTER(C.c_int)), ("nSubdomains", C.POINTER(C.c_int)),
                ("nSubdomainsProd", C.POINTER(C.c_int)), ("offset", C.POINTER(C.c_int)),
                ("posToSubdomain", C.POINTER(C.c_double)),
                ("nSpecies", C.c_int), ("nNeighbors", C.c_int), ("neighborhoodCenter", C.c_int),
                ("migrants", C.c_void_p), ("migrantsDummy", C.c_void_p),
                ("nEmigrants", C.POINTER(C.c_long)), ("nEmigrantsAlloc", C.POINTER(C.c_long)),
                ("nImmigrants", C.POINTER(C.c_long)), ("nImmigrantsAlloc", C.c_long),
                ("emigrants", C.c_void_p), ("emigrantsDummy", C.c_void_p), ("immigrants", C.c_void_p),
                ("thresholds", C.POINTER(C.c_double)), ("send", C.c_void_p), ("recv", C.c_void_p),
                ("comm", C.c_void_p)]


def test_neighbor_maps_known_answers(lib):
    """testPuRankNeighbor (test/pusher.test.c:549-573) on the product's
    puNeighborToRank / puRankToNeighbor / puNeighborToReciprocal."""
    k = GOLD["puRankNeighbor"]
    h = lib.HOST
    sub = (C.c_int * 3)(*k["subdomain"])
    ns = (C.c_int * 3)(*k["nSubdomains"])
    prod = (C.c_int * 4)(1, 5, 20, 60)
    m = MpiInfo(mpiRank=24, mpiSize=60, nDims=3, subdomain=sub, nSubdomains=ns, nSubdomainsProd=prod)
    h.puNeighborToRank.argtypes = [C.POINTER(MpiInfo), C.c_int]
    h.puRankToNeighbor.argtypes = [C.POINTER(MpiInfo), C.c_int]
    for ne, rank in k["neighbor_to_rank"].items():
        assert h.puNeighborToRank(C.byref(m), int(ne)) == rank
    for rank, ne in k["rank_to_neighbor"].items():
        assert h.puRankToNeighbor(C.byref(m), int(rank)) == ne
    for ne, rec in k["reciprocal_3d"].items():
        assert h.puNeighborToReciprocal(int(ne), 3) == rec


def test_neighbor_maps_match_oracle_exhaustive(lib):
    import orc
    o = orc._load()
    h = lib.HOST
    h.puNeighborToRank.argtypes = [C.POINTER(MpiInfo), C.c_int]
    h.puRankToNeighbor.argtypes = [C.POINTER(MpiInfo), C.c_int]
    rng = np.random.default_rng(3)
    for _ in range(20):
        nsv = rng.integers(1, 5, size=3).astype(np.int32)
        subv = np.array([rng.integers(0, n) for n in nsv], dtype=np.int32)
        ns = (C.c_int * 3)(*nsv.tolist())
        sub = (C.c_int * 3)(*subv.tolist())
        prod = (C.c_int * 4)(1, int(nsv[0]), int(nsv[0] * nsv[1]), int(nsv.prod()))
        m = MpiInfo(nDims=3, subdomain=sub, nSubdomains=ns, nSubdomainsProd=prod)
        for ne in range(27):
            assert h.puNeighborToRank(C.byref(m), ne) == o.orc_kat_neighbor_to_rank(
                nsv.ctypes.data_as(C.c_void_p), subv.ctypes.data_as(C.c_void_p), ne)
        for r in range(int(nsv.prod())):
            assert h.puRankToNeighbor(C.byref(m), r) == o.orc_kat_rank_to_neighbor(
                nsv.ctypes.data_as(C.c_void_p), subv.ctypes.data_as(C.c_void_p), r)


@pytest.mark.parametrize("name", ["langmuir1d", "langmuir2d", "cold3d", "warm"])
def test_ini_and_units_match_oracle(lib, name):
    """uAlloc + uNormalize (units.c) on the product side produce the same
    normalised charge, mass, time step and step size as the oracle."""
    import orc
    from pinc_amd import configs
    h = lib.HOST
    h.iniFromString.restype = C.c_void_p
    h.iniFromString.argtypes = [C.c_char_p]
    h.uAlloc.restype = C.c_void_p
    h.uAlloc.argtypes = [C.c_void_p]
    h.uNormalize.argtypes = [C.c_void_p, C.c_void_p]
    h.uFree.argtypes = [C.c_void_p]
    h.iniClose.argtypes = [C.c_void_p]
    h.iniGetDoubleArr.restype = C.POINTER(C.c_double)
    h.iniGetDoubleArr.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
    h.iniGetInt.argtypes = [C.c_void_p, C.c_char_p]
    kw = {"true_size": (32, 32, 32), "ppc": 1} if name == "warm" else {}
    cfg = configs.config(name, **kw)
    text = configs.to_ini(cfg)
    d = h.iniFromString(text.encode())
    u = h.uAlloc(d)
    h.uNormalize(d, u)
    ns = h.iniGetInt(d, b"population:nSpecies")
    charge = h.iniGetDoubleArr(d, b"population:charge", ns)
    mass = h.iniGetDoubleArr(d, b"population:mass", ns)
    ini = configs.write_ini(cfg)
    try:
        w = orc.World(ini)
        q_o, m_o = w.species()
        w.close()
    finally:
        Path(ini).unlink()
    for s in range(ns):
        assert charge[s] == q_o[s], (s, charge[s], q_o[s])
        assert mass[s] == m_o[s], (s, mass[s], m_o[s])
    h.uFree(u)
    h.iniClose(d)


def test_bench_config_sort_spread():
    """The opt-in spread gate of the adaptive sort reaches the ini only when
    asked for (population:sortSpread; the default schedule is unchanged)."""
    from pinc_amd import configs
    base = configs.bench_config("c4ts", 32, 4)
    assert "sortSpread" not in base["population"]
    assert base["population"]["sortFraction"] == "0.8"
    gated = configs.bench_config("c4ts", 32, 4, sort_spread=2.0)
    assert gated["population"]["sortSpread"] == "2.0"
    assert "sortSpread" not in configs.bench_config("c4", 32, 4, layout="reference")["population"]


@pytest.mark.parametrize("nb", [1, 7, 512, 513, 1048576, 1048576 + 300])
def test_push_chunk_placement_is_a_bijection(lib, nb):
    """The push's chunk -> XCD placement (push_chunk_of, shared by the kernel
    and the trace's per-XCD attribution): every chunk is taken by
    exactly one block and each XCD gets its share (host function, no GPU)."""
    xcd = np.full(nb, -1, dtype=np.int32)
    lib.HIP.pinc_hip_push_xcd_of_chunks.argtypes = [C.c_long, C.c_void_p]
    assert lib.HIP.pinc_hip_push_xcd_of_chunks(nb, xcd.ctypes.data) == 0
    assert xcd.min() >= 0 and xcd.max() <= 7
    counts = np.bincount(xcd, minlength=8)
    assert counts.max() - counts.min() <= 1, counts


class _Lvl(C.Structure):
    _fields_ = [("nd", C.c_int), ("T", C.c_int * 3)]


@pytest.mark.parametrize("case", ["3d", "odd_x", "too_many", "not_halving", "spectral_not_square", "cycles"])
def test_small_solve_rejects_bad_levels(lib, case):
    """pinc_hip_mg_solve_small checks its levels on the host before any
    launch (no GPU needed): a 3-D level, an x extent that is not a power of
    two, more than 16384 points, levels that do not halve, a non-square
    level 1 with the spectral basis, a cycle cap below 1 -- each returns a
    nonzero code and names itself in pinc_hip_error_string."""
    h = lib.HIP
    vp = C.c_void_p
    h.pinc_hip_mg_solve_small.argtypes = [vp, vp, vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                          vp, vp, vp]
    h.pinc_hip_error_string.restype = C.c_char_p
    shapes = {"3d": [(3, 16, 16, 16), (3, 8, 8, 8)], "odd_x": [(2, 96, 64, 1), (2, 48, 32, 1)],
              "too_many": [(2, 256, 128, 1), (2, 128, 64, 1)], "not_halving": [(2, 128, 128, 1), (2, 32, 64, 1)],
              "spectral_not_square": [(2, 128, 64, 1), (2, 64, 32, 1)], "cycles": [(2, 128, 128, 1), (2, 64, 64, 1)]}
    lv = shapes[case]
    arr = (_Lvl * len(lv))(*[_Lvl(nd, (C.c_int * 3)(a, b, c)) for nd, a, b, c in lv])
    basis = C.c_void_p(1) if case == "spectral_not_square" else None  # never dereferenced: rejected first
    cycles = 0 if case == "cycles" else 10
    rc = h.pinc_hip_mg_solve_small(None, None, None, len(lv), arr, 4, 4, 10, cycles, 1e-10, basis, None, None)
    assert rc != 0
    assert b"mg_solve_small" in h.pinc_hip_error_string()
