"""tools/kernel_gaps.py (CPU): idle time between kernels from a rocpd-style
database, on a synthetic trace of two steps with a known gap per pair."""
import sqlite3
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _trace(path: Path):
    # per step: efield, push (species 0), push (species 1), read (copy), solve kernel
    c = sqlite3.connect(path)
    c.execute("create table kernels (name text, start integer, end integer)")
    t = 0
    rows = []
    for _ in range(4):
        for name, dur, gap in (("void k_efield<3>(Args)", 100, 0), ("void (anonymous namespace)::k_push<3>(PushArgs)", 20000, 5000),
                               ("void (anonymous namespace)::k_push<3>(PushArgs)", 20000, 2000),
                               ("__amd_rocclr_copyBuffer", 5, 1000), ("void k_gs_sweep4c<32, 8, 256>(double*)", 170, 40000)):
            t += gap
            rows.append((name, t, t + dur))
            t += dur
    c.executemany("insert into kernels values (?, ?, ?)", rows)
    c.commit()
    c.close()


def test_gaps_by_pair_and_step(tmp_path):
    _trace(tmp_path / "run_results.db")
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "kernel_gaps.py"), str(tmp_path), "10"],
                         capture_output=True, text=True, check=True).stdout
    # the 40 us gap before each sweep follows the host read
    line = next(ln for ln in out.splitlines() if ln.startswith("__amd_rocclr_copyBuffer -> k_gs_sweep4c"))
    assert line.split()[-3:] == ["4", "40.0", "0.160"]
    # kernel names without the anonymous namespace prefix
    assert any(ln.startswith("k_push<3> -> k_push<3>") for ln in out.splitlines())
    # whole steps: 5 + 2 + 1 + 40 us idle of an 88.275 us step
    step = next(ln for ln in out.splitlines() if ln.startswith("whole steps"))
    assert "median idle 0.048 ms of a 0.088 ms step" in step, step
