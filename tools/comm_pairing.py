#!/usr/bin/env python3
"""Check the collectives every rank issued (PINC_COMM_TRACE logs,
pinc_amd/host/pinc_comm.c) against RCCL's matching rules.

    python tools/comm_pairing.py <trace_dir> [<world_size>]

RCCL (as NCCL) needs
  * every rank to issue the same collectives (allgather "G", allreduce "R")
    in the same order with the same element counts, and the grouped
    point-to-point exchanges ("X") at the same places in that order: a rank
    that skips or reorders one hangs the job instead of failing;
  * inside an exchange, the k-th send from rank a to rank b to meet the k-th
    receive posted by b from a (per ordered pair, in issue order, zero-byte
    operations are not posted) with the same byte count.  The host transport
    (gloo) of the rehearsals matches by tag instead, so a pairing that only
    tags make right would pass there and hang under RCCL; this check applies
    RCCL's rule to the sequence the rehearsal recorded.

Exit status 0 and a summary when everything pairs, 1 with the first
mismatches otherwise.
"""
from __future__ import annotations

import re
import sys
from collections import Counter
from pathlib import Path


def parse(path: Path) -> list:
    ops = []
    for line in path.read_text().splitlines():
        kind, seq, rest = line.split(" ", 2)
        label, _, tail = rest.partition("|")
        if kind == "X":
            f = tail.split()
            n = int(f[0])
            sends, recvs = [], []
            for i in range(n):
                sp, sb = re.fullmatch(r"s(-?\d+):(\d+)", f[1 + 2 * i]).groups()
                rp, rb = re.fullmatch(r"r(-?\d+):(\d+)", f[2 + 2 * i]).groups()
                sends.append((int(sp), int(sb)))
                recvs.append((int(rp), int(rb)))
            ops.append(("X", label, sends, recvs))
        else:
            ops.append((kind, label, int(tail)))
    return ops


def load(d: Path) -> dict:
    traces = {}
    for f in sorted(d.glob("comm_rank*.log")):
        traces[int(re.search(r"comm_rank(\d+)\.log", f.name).group(1))] = parse(f)
    return traces


def check(traces: dict, world: int | None = None, max_errors: int = 20) -> tuple[list, dict]:
    errs = []
    ranks = sorted(traces)
    if world is not None and ranks != list(range(world)):
        errs.append(f"trace files for ranks {ranks}, expected 0..{world - 1}")
        return errs, {}
    P = len(ranks)
    lens = {r: len(traces[r]) for r in ranks}
    if len(set(lens.values())) != 1:
        errs.append(f"ranks issued different numbers of collectives: {lens}")
    n = min(lens.values()) if lens else 0
    stats = Counter()
    for i in range(n):
        head = [(traces[r][i][0], traces[r][i][1]) for r in ranks]
        if len(set(head)) != 1:
            errs.append(f"collective #{i}: ranks disagree on what comes next: {dict(zip(ranks, head))}")
            break
        kind, label = head[0]
        stats[(kind, label)] += 1
        if kind in "GR":
            counts = {r: traces[r][i][2] for r in ranks}
            if len(set(counts.values())) != 1:
                errs.append(f"collective #{i} {kind} '{label}': element counts differ {counts}")
            continue
        # exchange: per ordered pair, the nonzero sends of a to b in issue
        # order must equal the nonzero receives of b from a in issue order
        for a in ranks:
            for b in ranks:
                snd = [by for (p, by) in traces[a][i][2] if p == b and by > 0]
                rcv = [by for (p, by) in traces[b][i][3] if p == a and by > 0]
                if snd != rcv:
                    errs.append(f"collective #{i} exchange '{label}': rank {a} sends {snd} B to rank {b}, "
                                f"which posts receives of {rcv} B from rank {a}")
        for a in ranks:
            for (p, _), (q, _) in zip(traces[a][i][2], traces[a][i][3]):
                if not (0 <= p < P and 0 <= q < P):
                    errs.append(f"collective #{i} exchange '{label}': rank {a} names peer {p}/{q} outside 0..{P - 1}")
        if len(errs) >= max_errors:
            break
    return errs[:max_errors], dict(stats)


def main() -> int:
    d = Path(sys.argv[1])
    world = int(sys.argv[2]) if len(sys.argv) > 2 else None
    traces = load(d)
    errs, stats = check(traces, world)
    if errs:
        print("\n".join(errs))
        return 1
    n = len(next(iter(traces.values()))) if traces else 0
    print(f"{len(traces)} ranks, {n} collectives each, all paired under RCCL's rules:")
    for (kind, label), c in sorted(stats.items(), key=lambda kv: -kv[1]):
        print(f"  {kind} {label}: {c}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
