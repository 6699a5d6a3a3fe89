"""The hot kernels keep their registers (CPU: the compiler's resource report,
written by pinc_amd/build.py next to the libraries).

Spilled VGPRs are scratch traffic in HBM.  In round 4 a change to the
counting code spilled 52 VGPRs in the plain push and cost 4 ms per launch,
with correct results.  A change that spills the push, the smoother or the
level transfers fails here, at build time, instead of in the next bench.
"""
import pytest

from pinc_amd import build

# kernels (substring of the mangled name) that must not spill, and the
# least waves per SIMD they are designed for
HOT = {
    "k_pushILi3E": 4,           # every 3-D fused push instance (plain / count / sort, objects)
    "k_gs_sweep4cILi32ELi8ELi256E": 2,  # (round 5: phi and rho rings, 80 KB of LDS: two workgroups per CU)
    "k_gs_sweep2ILi32ELi8ELi256E": 1,
    "k_resid_restrict3": 1,
    "k_prolong_add3c": 1,
    "k_residual_sumsq": 1,
    "k_deposit_tiled": 1,
}


def test_resource_reports_present(built):
    res = build.kernel_resources()
    assert res, "no resource reports next to the libraries (pinc_amd/build.py)"
    for key in HOT:
        assert any(key in k for k in res), key


@pytest.mark.parametrize("key", sorted(HOT))
def test_hot_kernels_do_not_spill(built, key):
    res = build.kernel_resources()
    hits = {k: v for k, v in res.items() if key in k}
    assert hits, key
    for k, v in hits.items():
        assert v.get("vgpr_spill", 0) == 0, (k, v)
        assert v.get("occupancy", 0) >= HOT[key], (k, v)
