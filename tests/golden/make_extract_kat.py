#!/usr/bin/env python3
"""Adds the `extractEmigrantsXD` known answer to reference_outputs.json.

Restates, as data, the inputs and expectations of the reference's
testExtractEmigrantsXD (test/pusher.test.c:360-545), which pins the serial
back-fill order of puExtractEmigrants3D/ND (src/pusher.c:782-910):

  * 3 species, nAlloc 100 each (iStart 0, 100, 200), trueSize 8^3, one ghost
    layer, nEmigrantsAlloc 10;
  * species 0 and 1 each get (pNew, in this order) a line of 21 particles at
    x = 0, 0.5, ..., 10 (y = z = 5), then one particle in each of the 27
    regions at 5 + 4.5 (x, y, z), x fastest; velocity (1, 2, 3) for all;
    species 2 stays empty;
  * expected: the 81 emigrant counts (ne * nSpecies + s), the records of
    emigrants[12] and emigrants[14] in buffer order, one record per species of
    every other direction, iStop = {17, 117, 200}, and the 17 survivors of each
    species in slot order.

Restatement: the test sets grid:thresholds = 1,1,1,-1,-1,-1 for the upper
rule it was written against.  The current gAllocMpi counts upper thresholds
from the upper edge, upper = (size - 1) - thr (src/grid.c:1094-1099, size = 10
with the ghosts), so the same lower 1 and upper 9 are thresholds 1,1,1,0,0,0
now -- the same kind of restatement as the gCreateNeighborhood entry.  (With
the literal -1 the upper threshold would be 10 and the expected counts, which
the test asserts, could not hold: 9 and 9.5 would stay.)

    python tests/golden/make_extract_kat.py     # rewrites the entry in place
"""
import json
from pathlib import Path

HERE = Path(__file__).resolve().parent
OUT = HERE / "reference_outputs.json"


def particles():
    """pNew order of one species (both species get the same list)."""
    pos = []
    x = 0.0
    while x <= 10:
        pos.append([x, 5.0, 5.0])
        x += 0.5
    for z in (-1, 0, 1):
        for y in (-1, 0, 1):
            for x in (-1, 0, 1):
                pos.append([5 + x * 4.5, 5 + y * 4.5, 5 + z * 4.5])
    return pos


def entry():
    vel = [1.0, 2.0, 3.0]
    counts = [1, 1, 0] * 27
    counts[12 * 3:12 * 3 + 3] = [3, 3, 0]
    counts[13 * 3:13 * 3 + 3] = [0, 0, 0]
    counts[14 * 3:14 * 3 + 3] = [4, 4, 0]
    rec = lambda x: [x, 5.0, 5.0] + vel
    buffers = {
        "12": [rec(x) for x in (0.0, 0.5, 0.5, 0.0, 0.5, 0.5)],
        "14": [rec(x) for x in (9.5, 10.0, 9.5, 9.0, 9.5, 10.0, 9.5, 9.0)],
    }
    for z in (-1, 0, 1):
        for y in (-1, 0, 1):
            for x in (-1, 0, 1):
                ne = (x + 1) + (y + 1) * 3 + (z + 1) * 9
                if ne < 12 or ne > 14:
                    r = [5 + x * 4.5, 5 + y * 4.5, 5 + z * 4.5] + vel
                    buffers[str(ne)] = [r, r]
    survivors = [5.0, 8.5] + [1.0 + 0.5 * k for k in range(15)]
    return {
        "source": "test/pusher.test.c:360-545 (thresholds restated for the current upper = (size-1) - thr "
                  "rule, src/grid.c:1094-1099: the test's 1,1,1,-1,-1,-1 give lower 1 and upper 9 under the rule "
                  "it was written for, which is 1,1,1,0,0,0 now)",
        "ini": {"grid:trueSize": "8,8,8", "grid:nGhostLayers": "1", "grid:nSubdomains": "1,1,1",
                "grid:thresholds": "1,1,1,0,0,0", "grid:nEmigrantsAlloc": "10",
                "population:nAlloc": "100,100,100", "population:charge": "-1,1,2", "population:mass": "10,1,10"},
        "thresholds_ini_test": [1, 1, 1, -1, -1, -1],
        "expect_thresholds": [1.0, 1.0, 1.0, 9.0, 9.0, 9.0],
        "iStart": [0, 100, 200],
        "pos": particles(),
        "vel": vel,
        "species_with_particles": [0, 1],
        "expect_nEmigrants": counts,
        "expect_emigrants": buffers,
        "expect_iStop": [17, 117, 200],
        "expect_survivor_x": survivors,
        "survivor_yz": [5.0, 5.0],
    }


def main():
    d = json.loads(OUT.read_text())
    d["kat"]["extractEmigrantsXD"] = entry()
    OUT.write_text(json.dumps(d, indent=1) + "\n")


if __name__ == "__main__":
    main()
