"""The struct ABI against the reference's core.h.

tests/golden/core_layout.json holds the field order, declared types and
LP64 offsets of Population (core.h:72-86), MpiInfo (:112-138), Grid
(:261-277), Units (:392-417) and Timer (:439-442), extracted from the
reference's header text by tests/golden/make_core_layout.py.  A probe
compiled against include/core.h (the forwarding header main.c:10 includes)
prints offsetof and sizeof of every field; each must equal the reference's.
The device twins this build appends must come after the reference's last
field.  CPU only (gcc).
"""
import json
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LAYOUT = json.loads((ROOT / "tests" / "golden" / "core_layout.json").read_text())
APPENDED = {"Population": ["dev"], "MpiInfo": ["comm"], "Grid": ["dev"], "Units": [], "Timer": []}


def _probe(tmp_path, headers=("core.h", "pusher.h", "multigrid.h", "spectral.h")) -> dict:
    lines = [f'#include "{h}"' for h in headers]
    lines += ["#include <stddef.h>", "int main(void){"]
    for s, v in LAYOUT["structs"].items():
        lines.append(f'printf("%s __sizeof__ %zu\\n", "{s}", sizeof({s}));')
        for f in v["fields"] + [{"name": n} for n in APPENDED[s]]:
            n = f["name"]
            lines.append(f'printf("%s %s %zu %zu\\n", "{s}", "{n}", offsetof({s}, {n}), sizeof((({s} *)0)->{n}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)],
                   check=True)
    out = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        p = line.split()
        if p[1] == "__sizeof__":
            out[(p[0], None)] = int(p[2])
        else:
            out[(p[0], p[1])] = (int(p[2]), int(p[3]))
    return out


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    return _probe(tmp_path_factory.mktemp("layout"))


@pytest.mark.parametrize("struct", list(LAYOUT["structs"]))
def test_reference_fields_at_reference_offsets(probe, struct):
    v = LAYOUT["structs"][struct]
    for f in v["fields"]:
        got = probe[(struct, f["name"])]
        assert got == (f["offset"], f["size"]), (struct, f["name"], f["type"], got, (f["offset"], f["size"]))


@pytest.mark.parametrize("struct", list(LAYOUT["structs"]))
def test_device_twins_appended_after_the_reference_fields(probe, struct):
    v = LAYOUT["structs"][struct]
    end = v["fields"][-1]["offset"] + v["fields"][-1]["size"]
    for n in APPENDED[struct]:
        assert probe[(struct, n)][0] >= end, (struct, n)
    if not APPENDED[struct]:
        assert probe[(struct, None)] == v["size"], struct


def test_timer_total_first():
    """main.c:276 prints tMsg(t->total, ...): total is core.h's first Timer
    field."""
    assert [f["name"] for f in LAYOUT["structs"]["Timer"]["fields"]] == ["total", "start"]


def test_reference_header_names_compile_standalone(tmp_path):
    """Each of main.c's four includes works on its own (the C driver uses
    all four, tests/c_driver/pinc_mainc.c)."""
    for h in ("core.h", "pusher.h", "multigrid.h", "spectral.h"):
        p = _probe(tmp_path, headers=(h,))
        assert p[("Timer", "total")] == (0, 8)
