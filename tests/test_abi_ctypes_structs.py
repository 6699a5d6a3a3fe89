"""The ctypes mirrors the GPU tests pass to the C ABI have the size and
field offsets of the structs in include/pinc_hip.h (CPU: a gcc probe).

A field added to pinc_push_t but not to its ctypes mirror makes the kernel
read the pointers after the mirror's end: a GPU fault in the test, not a
failed assertion.  This test catches it on the CPU first.
"""
import ctypes as C
import importlib.util
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
KAT = Path(__file__).parent / "test_gpu_reference_kat.py"


def _mirrors():
    spec = importlib.util.spec_from_file_location("kat_mirrors", KAT)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return {"pinc_push_t": m.PushArgs, "pinc_pop_t": m.Pop, "pinc_geom_t": m.Geom}


def _probe(tmp_path, structs):
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "pinc_hip.h"', "int main(void) {"]
    for name, cls in structs.items():
        lines.append(f'  printf("{name} __sizeof__ %zu\\n", sizeof({name}));')
        for f in cls._fields_:
            lines.append(f'  printf("{name} {f[0]} %zu\\n", offsetof({name}, {f[0]}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)], check=True)
    out = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        s, f, v = line.split()
        out[(s, f)] = int(v)
    return out


def test_ctypes_mirrors_match_the_header(tmp_path):
    structs = _mirrors()
    got = _probe(tmp_path, structs)
    for name, cls in structs.items():
        assert C.sizeof(cls) == got[(name, "__sizeof__")], (name, C.sizeof(cls), got[(name, "__sizeof__")])
        for f in cls._fields_:
            assert getattr(cls, f[0]).offset == got[(name, f[0])], (name, f[0])
