"""Generate tests/golden/core_layout.json: the field order, C types and LP64
offsets of the reference's core structs.

Run in the survey container only (it reads /root/reference/src/core.h as
text; the GPU box has no /root/reference).  The JSON is data: for each of
Population (core.h:72-86), MpiInfo (:112-138), Grid (:261-277), Units
(:392-417) and Timer (:439-442), every field in declaration order with its
declared type, and the offset and size it has under the x86-64 / LP64 ABI
(which the host library is built for), with

  * hid_t = int64_t (HDF5 >= 1.10; the library loads HDF5 at run time),
  * MPI_Request * and bndType * = pointers, enums = 4 bytes.

tests/test_core_layout.py compiles a probe against include/core.h and checks
offsetof and sizeof of every field against this file.

    python tests/golden/make_core_layout.py [path/to/core.h]
"""
import json
import re
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/core.h")
STRUCTS = ("Population", "MpiInfo", "Grid", "Units", "Timer")

SCALARS = {"int": 4, "long int": 8, "long": 8, "double": 8, "unsigned long long int": 8,
           "unsigned long long": 8, "hid_t": 8, "bool": 1, "bndType": 4}


def parse(text: str) -> dict:
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    out = {}
    for m in re.finditer(r"typedef\s+struct\s*\{(.*?)\}\s*(\w+)\s*;", text, flags=re.S):
        name = m.group(2)
        if name not in STRUCTS:
            continue
        fields = []
        for decl in m.group(1).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            # "double *pos" / "int *subdomain" / "long int **migrants"
            dm = re.match(r"^(.*?)((?:\*\s*)*)(\w+)$", decl)
            base, stars, fname = dm.group(1).strip(), dm.group(2).replace(" ", ""), dm.group(3)
            fields.append({"name": fname, "type": base + (" " + stars if stars else "")})
        out[name] = fields
    return out


def layout(fields: list) -> tuple[list, int]:
    off, align_max = 0, 1
    res = []
    for f in fields:
        t = f["type"]
        if "*" in t:
            size = 8
        else:
            size = SCALARS[t]
        align = size
        off = (off + align - 1) // align * align
        res.append(dict(f, offset=off, size=size))
        off += size
        align_max = max(align_max, align)
    total = (off + align_max - 1) // align_max * align_max
    return res, total


def main() -> int:
    structs = parse(SRC.read_text())
    missing = [s for s in STRUCTS if s not in structs]
    if missing:
        raise SystemExit(f"not found in {SRC}: {missing}")
    data = {"source": "src/core.h", "abi": "x86-64 LP64, hid_t = int64_t", "structs": {}}
    for s in STRUCTS:
        fields, total = layout(structs[s])
        data["structs"][s] = {"size": total, "fields": fields}
    (HERE / "core_layout.json").write_text(json.dumps(data, indent=1) + "\n")
    for s in STRUCTS:
        print(s, data["structs"][s]["size"], [f["name"] for f in data["structs"][s]["fields"]])
    return 0


if __name__ == "__main__":
    sys.exit(main())
