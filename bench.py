#!/usr/bin/env python3
"""bench.py -- PINC per-timestep PIC hot path on MI355X.

Workload (BASELINE.json metric "particle-updates/sec + Poisson-solve
ms/step, 256^3 grid 64 ppc, 1/2/4/8 MI355X"): the warm 3-D two-species plasma
of config C4 (warm_big.ini family) on a 256^3 periodic grid
with 64 particles per cell per species (2.15 G particles), Maxwellian
velocities (v_th,e = 0.05 cells/step) from the counter RNG, decomposed into
N slabs along z for N GPUs (strong scaling: the global problem is fixed).
One step = move + migrate + deposit + multigrid solve + E field + accelerate,
i.e. main.c:197-274.  The solve runs in native mode by default: the
reference's own mgVRecursive does not converge on this grid (DESIGN.md
section 6; --mg reference runs it anyway).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints one JSON line.  value = particles x K / (max over ranks of the
K-step wall time).  Every probed kernel's launches inside the timed region
are timed with HIP events on the library's stream; `roofline` reports the
one with the most time per step, `kernels` all of them.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# the measured copy ceiling of the push's own streams (six SoA arrays, each a
# separate allocation, one block per 1024-particle chunk, nontemporal):
# profiles/r05e_copy_ceiling.json (tools/copy_probe2.hip)
COPY_CEILING = ROOT / "profiles" / "r05e_copy_ceiling.json"


def _copy_ceiling_gbs() -> float | None:
    try:
        return 1000.0 * json.loads(COPY_CEILING.read_text())["push_streams_ceiling_TBs"]
    except (OSError, ValueError, KeyError, TypeError):
        return None
METRIC = "particle-updates/sec + Poisson-solve ms/step, 256³ grid 64 ppc, 1/2/4/8 MI355X"
# kernel names as rocprofv3 --kernel-trace reports them (3-D instantiations)
ROCPROF_NAMES = {
    "gs_pass": "k_gs_pass<3, true>",
    "accelerate": "k_accel<3, true, true>",
    "move_classify": "k_move_classify<3>",
    "deposit": "k_deposit_tiled<3, true>",
    "residual_sumsq": "k_residual_sumsq3p",
    "mg_cycle": "one V-cycle, replayed as a HIP graph (all levels)",
}


def _pmc_traffic(prefix: str, key: dict):
    """HBM bytes per launch of the kernels whose rocprof name starts with
    `prefix`, from the newest profiles/*_hbm_traffic.json whose "config"
    (written by tools/pmc_summary.py from the profiled bench line) is this
    run's configuration `key` (workload, grid, ppc, GPU count, layout),
    launch-weighted over the kernel's variants; None if no profile of this
    configuration covers it."""
    def order(f):  # round, then tag: r03w < r03ao < r04a (tags grow a letter once z is used)
        m = re.match(r"r(\d+)([a-z]*)_", f.name)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, f.name)

    files = sorted((ROOT / "profiles").glob("*_hbm_traffic.json"), key=order)
    for f in reversed(files):
        try:
            d = json.loads(f.read_text())
            ks = d["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        if d.get("config") != key:
            continue
        sel = [k for k in ks if k["name"].startswith(prefix) and k.get("traffic_bytes_per_launch_mean")
               and k["grid_size"] >= 1 << 20]
        if sel:
            n = sum(k["launches"] for k in sel)
            t = sum(k["traffic_bytes_per_launch_mean"] * k["launches"] for k in sel) / n
            return {"bytes_per_launch": t, "source": f.name, "launches": n,
                    "fetch_correction": sel[0].get("fetch_correction"), "calibration": d.get("calibration")}
    return None


def _host_cpus() -> dict:
    """The host CPUs this process owns: its affinity set, capped by the
    cgroup's CPU quota where one is set (cpu.max: a box may pin a job to
    many CPUs but grant it the time of fewer).  PINC_CPU_THREADS overrides."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    if os.environ.get("PINC_CPU_THREADS"):
        threads = max(1, int(os.environ["PINC_CPU_THREADS"]))
    return {"threads": threads, "affinity": aff, "cgroup_quota_cpus": quota, "nproc": os.cpu_count()}


def _mem_available() -> int:
    try:
        for line in Path("/proc/meminfo").read_text().splitlines():
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def _cpu_baseline(size: int, ppc: int, steps: int, native: bool, workload: str = "c4",
                  extrapolate: int = 0, spectral_coarse: int = 0, size_note: str = "") -> dict:
    """The oracle (plain-C restatement of the reference) on the host cores,
    on a bounded sample of the same workload: the warm plasma at size^3 with
    ppc particles per cell per species, decomposed into one z-slab per
    thread (grid:nSubdomains = 1,1,T, the reference's MPI decomposition,
    emulated ranks in parallel with OpenMP), solving with the same multigrid
    algorithm as the GPU line (native mode, orc_native.c, or the
    reference's)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import orc  # test/baseline infrastructure only
    from pinc_amd import configs
    cpus = _host_cpus()
    threads = cpus["threads"]
    nsub = threads
    while nsub > 1 and (size % nsub or (size // nsub) % 2):
        nsub -= 1
    orc.LIB.orc_set_threads(threads)
    nd = 2 if workload == "c2" else 3
    if workload == "c2":
        cfg = configs.config("c2")
        cfg["grid"]["trueSize"] = f"{size},{size // nsub}"
        cfg["grid"]["nSubdomains"] = f"1,{nsub}"
        cfg["population"]["nParticles"] = f"{ppc} pc"
        cfg["population"]["nAlloc"] = f"{ppc + 16} pc"
        cfg["multigrid"]["mgLevels"] = "1" if native else cfg["multigrid"]["mgLevels"]
    else:
        cfg = configs.config({"c3": "c3", "c4ts": "c4ts"}.get(workload, "warm"), true_size=(size, size, size // nsub),
                             nsub=(1, 1, nsub), ppc=ppc, nalloc_pc=ppc + 8, levels=1 if native else 5)
    if native and cfg["methods"]["poisson"] == "mgSolver":
        cfg["multigrid"]["native"] = "1"
        cfg["multigrid"]["extrapolate"] = str(extrapolate)
        cfg["multigrid"]["spectralCoarse"] = str(spectral_coarse)
    ini = configs.write_ini(cfg)
    t_init = time.perf_counter()
    w = orc.World(ini)
    w.init(perturb=workload == "c2", maxwell=workload != "c2", seed=20260101)
    w.init_fields()
    t_init = time.perf_counter() - t_init
    ns = int(cfg["population"]["nSpecies"])
    n = sum(w.count(s, rank=r) for r in range(w.nranks) for s in range(ns))
    c0 = w.cycles
    ph0 = w.timers()
    t0 = time.perf_counter()
    w.step(steps)
    dt = time.perf_counter() - t0
    ph = {k: (v - ph0[k]) * 1e3 / steps for k, v in w.timers().items()}
    cyc = (w.cycles - c0) / steps
    levels = orc.LIB.orc_world_mg_levels(w._h)
    w.close()
    os.unlink(ini)
    push_ms = ph["move"] + ph["migrate"] + ph["deposit"] + ph["accelerate"]
    return {"value": n * steps / dt, "unit": "particle-updates/s", "cores": threads, "kind": "port",
            "nproc": cpus["nproc"], "cpu_affinity": cpus["affinity"], "cgroup_quota_cpus": cpus["cgroup_quota_cpus"],
            "sample": f"oracle (C restatement of the reference, OpenMP over {nsub} emulated slab ranks, "
                      f"{threads} threads = the CPUs this process owns) on the same {workload.upper()} workload at "
                      f"{size}^{nd}{size_note}, {ppc} ppc x {ns} species ({n} particles), {steps} steps; "
                      + ("spectral solve (naive DFT restatement)" if cfg["methods"]["poisson"] == "sSolver" else
                         "multigrid " + ("native mode as the GPU line" + (" (extrapolated initial guess)"
                                                                           if extrapolate else "")
                                         + (" (level 1 solved exactly by DFT)" if spectral_coarse else
                                            " (levels >= 1 recursively as a V-cycle: the GPU line solves level 1 "
                                            "exactly by FFT, same cycle count)" if native else "")
                                         if native else "reference algorithm")
                         + f", {levels} levels, {cyc:.0f} V-cycles/solve"),
            "algorithm_note": "the CPU and GPU lines run the same discretisation and stopping rule; the GPU line's "
                              "solver extensions (exact level-1 solve by FFT, spectral second guess with objects) "
                              "have no FFT library on the CPU side, so value ratios compare algorithm + hardware",
            "seconds": dt, "init_s": t_init,
            "push_deposit_updates_per_s": n / (push_ms * 1e-3) if push_ms > 0 else None,
            "poisson_ms_per_step": ph["solve"], "mg_cycles_per_solve": cyc,
            "phase_ms_per_step": ph}


def _push_order(samples: list) -> list:
    """Per species, the fused push launches of the timed steps by kind
    (`_lib.probe_samples("push")`, launch order): mean plain, count and sort
    launch, the "fresh" plain launch (the first after each sort of that
    species, or the run's first), and the ratios the sort schedule is judged
    by -- the plain push's decay between sorts and the sorting push's cost."""
    names = ("plain", "count", "sort")   # _lib.PUSH_KIND_NAMES
    by = {}
    for ms, tag in samples:
        by.setdefault(tag & 0xff, []).append((ms, names[tag >> 8]))
    out = []
    for s in sorted(by):
        seq = by[s]
        kinds = {k: [m for m, kk in seq if kk == k] for k in names}
        fresh, after_sort = [], True
        for m, k in seq:
            if k == "plain" and after_sort:
                fresh.append(m)
            after_sort = k == "sort"
        mean = {k: (sum(v) / len(v) if v else None) for k, v in kinds.items()}
        f = sum(fresh) / len(fresh) if fresh else None
        row = {"species": s, "launches": len(seq), "sorts": len(kinds["sort"]), "counts": len(kinds["count"]),
               "plain_ms": mean["plain"], "count_ms": mean["count"], "sort_ms": mean["sort"], "fresh_plain_ms": f,
               "all_ms": sum(m for m, _ in seq) / len(seq)}
        if mean["plain"] and f:
            row["plain_vs_fresh"] = mean["plain"] / f
        for k in ("count", "sort"):
            if mean[k] and mean["plain"]:
                row[f"{k}_vs_plain"] = mean[k] / mean["plain"]
        out.append(row)
    return out


def _multi_rank_summary(info: list, steps: int, dom: str, transport: str) -> dict:
    """What an N-GPU line needs to say where the time went: every phase's
    maximum (and minimum) over the ranks, each collective kind's device time,
    payload bytes and calls per step (pinc_comm.c statistics; the maximum
    over the ranks), and each rank's roofline of the dominant kernel
    (algorithmic bytes per launch over its mean launch time)."""
    phases = sorted(info[0]["phase_ms"])
    out = {"transport": transport, "ranks": len(info),
           "phase_ms_per_step_max": {k: max(i["phase_ms"][k] for i in info) / steps for k in phases},
           "phase_ms_per_step_min": {k: min(i["phase_ms"][k] for i in info) / steps for k in phases}}
    comm = {}
    for kind in info[0]["comm"]:
        per = [i["comm"][kind] for i in info]
        # calls beyond the event pool are counted but not timed: scale
        ms = [c["ms"] * (c["calls"] / c["timed_calls"]) if c["timed_calls"] else 0.0 for c in per]
        comm[kind] = {"ms_per_step_max": max(ms) / steps, "ms_per_step_mean": sum(ms) / len(ms) / steps,
                      "bytes_per_step_per_rank_max": max(c["bytes"] for c in per) / steps,
                      "calls_per_step": max(c["calls"] for c in per) / steps}
    out["comm_per_step"] = comm
    out["comm_ms_per_step_max_total"] = sum(v["ms_per_step_max"] for v in comm.values())
    per_rank = []
    for i in info:
        p = i["probes"].get(dom)
        r = {"rank": i["rank"], "particles": i["particles"], "wall_s": i["wall_s"]}
        if p and p["mean_ms"] > 0:
            gbs = p["mean_bytes"] / (p["mean_ms"] * 1e-3) / 1e9
            r["roofline"] = {"kernel": dom, "bytes_per_launch": p["mean_bytes"], "mean_launch_ms": p["mean_ms"],
                             "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS, "launches": p["launches"]}
        per_rank.append(r)
    out["per_rank"] = per_rank
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c4", choices=["c4", "c3", "c5", "c2", "c4ts"],
                    help="c4: warm 3-D plasma, 256^3, 64 ppc, multigrid (BASELINE.json metric, default); "
                         "c4ts: C4's two-stream variant (two electron beams, drift +-0.1 cells/step per component, "
                         "plus ions, 43 ppc per species); "
                         "c3: Maxwellian 128^3, 32 ppc, spectral (rocFFT) Poisson solve; "
                         "c5: c4 plus an immersed sphere (object.c: charge collection in the fused push, "
                         "capacitance correction, second solve); "
                         "c2: input/langmuir2D.ini at 128^2, 32 ppc (Langmuir perturbation, cold), multigrid")
    ap.add_argument("--size", type=int, default=None, help="global cells per dimension (c4: 256, c3: 128)")
    ap.add_argument("--ppc", type=int, default=None, help="particles per cell per species (c4: 64, c3: 32)")
    ap.add_argument("--mg-graph", type=int, default=None,
                    help="1: native multigrid replays each V-cycle as a captured HIP graph (multigrid:graph); "
                         "default 1 for C2 (where --mg-one-cu, on by default, bypasses it), 0 elsewhere "
                         "(neutral at C4)")
    ap.add_argument("--mg-one-cu", type=int, default=None,
                    help="1: a native one-rank 2-D solve of at most 16384 points runs all its cycles and the "
                         "convergence test in one workgroup (multigrid:oneCU, pinc_hip_mg_solve_small; with "
                         "--mg-spectral-coarse the level-1 correction by the f64 matrix cores); default 1 for C2")
    ap.add_argument("--mg-spectral-coarse", type=int, default=1,
                    help="1: native multigrid solves level 1's correction exactly by FFT (multigrid:spectralCoarse) "
                         "instead of recursing to the coarser levels")
    ap.add_argument("--mg-extrapolate", type=int, default=1,
                    help="1: native multigrid starts each solve from 2 phi_n - phi_(n-1) instead of phi_n "
                         "(multigrid:extrapolate; with an object, the two solves of a step from their own histories)")
    ap.add_argument("--mg-smooth", default="4,4",
                    help="native multigrid: smoothing counts PRE,POST (multigrid:nPreSmooth/nPostSmooth; default "
                         "4,4, the measured best at C4: 4 two-grid cycles per solve instead of 3 at the ini's 10,10, "
                         "same 1e-10 stop; 'ini' keeps the ini's)")
    ap.add_argument("--mg", default="native", choices=["native", "reference"],
                    help="native: correction-scheme V-cycle with the coarse h^2 factor (default; the reference "
                         "algorithm does not converge at 256^3 with 5 levels, DESIGN.md section 6); reference: "
                         "the reference's mgVRecursive exactly")
    ap.add_argument("--mg-shard", default="auto", choices=["auto", "0", "1"],
                    help="native multigrid level 0 sharded over the z-slabs with a deep halo (DESIGN.md section 7): "
                         "auto (default: from the rank count at which the extended slab is at most half the grid, "
                         "4 at 256^3), 1 (whenever possible, also on one rank), 0 (replicated solve)")
    ap.add_argument("--layout", default="tiled", choices=["tiled", "reference"],
                    help="tiled: particles re-sorted by 4^3-cell tile every --sort-interval moves (default); "
                         "reference: the reference's particle order (bit-exact indices)")
    ap.add_argument("--obj-second-guess", default="spectral", choices=["response", "spectral"],
                    help="objects with --mg-extrapolate: the second solve of a step starts from the first solution "
                         "plus the last step's correction response, or plus the exact discrete response to this "
                         "step's correction charge (rocFFT)")
    ap.add_argument("--obj-capacitance", default="solve", choices=["solve", "green"],
                    help="c5: capacitance matrix by one solve per surface node (the reference's, default) or "
                         "by translating one periodic response (objects:capacitance = green)")
    ap.add_argument("--c5-fused", type=int, default=1, choices=[0, 1],
                    help="c5: 1 = collection in the fused push (default), 0 = the unfused operators")
    ap.add_argument("--sort-interval", type=int, default=8)
    ap.add_argument("--sort-fraction", type=float, default=0.8,
                    help="> 0: sort each species once this fraction of its particles left their cell since its "
                         "last sort (adaptive, per species; --sort-max pushes apart at most) instead of every "
                         "--sort-interval pushes")
    ap.add_argument("--sort-max", type=int, default=32)
    ap.add_argument("--sort-spread", type=float, default=0.0,
                    help="with --sort-fraction: a sort also waits until the blocks' mean input cell box has grown "
                         "to this multiple of its size right after the last sort (0: off)")
    ap.add_argument("--sort-in-push", type=int, default=1,
                    help="1: the tile sort rides in every sort-interval-th push (default); 0: separate sort pass")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-size", type=int, default=None,
                    help="CPU baseline grid (default: the GPU line's, if the host has the memory, else 128)")
    ap.add_argument("--cpu-steps", type=int, default=None, help="CPU baseline steps (default 3 at 256^3, 20 below)")
    ap.add_argument("--host-transport", action="store_true",
                    help="rehearsal only: N ranks share GPU 0 and the collectives go through the gloo host "
                         "transport (RCCL refuses two ranks on one device); never the measured configuration")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    # the result line goes to the real stdout; with several ranks, fd 1 is
    # pointed at stderr for everything else, because gloo's C++ layer prints
    # its connection messages to stdout (and flushes them at exit)
    out = sys.stdout
    if world > 1:
        sys.stdout.flush()
        out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)

    # PINC_TORCH_STACK=0 (one rank): no torch in the process, so the
    # libraries run on /opt/rocm's HIP runtime and rocFFT, as the C driver does
    torch_stack = os.environ.get("PINC_TORCH_STACK", "1") != "0"
    if not torch_stack and world > 1:
        raise SystemExit("PINC_TORCH_STACK=0 runs one rank (torch.distributed is the control plane)")
    if args.host_transport:
        local = 0
    if torch_stack:
        import torch
        torch.cuda.set_device(local)

    def device_sync():
        if torch_stack:
            torch.cuda.synchronize()
    dist = None
    if world > 1:
        # control plane only (barriers, the communicator id, max-over-ranks
        # timing): gloo over TCP.  The data path is the library's own RCCL
        # communicator (pinc_hip_comm_init), so torch's bundled RCCL is never
        # brought up next to it.
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    red_dev = "cpu"

    from pinc_amd import configs, _lib
    from pinc_amd.sim import Sim

    comm_id = None
    transport = None
    if world > 1 and args.host_transport:
        from pinc_amd.transport import GlooTransport
        transport = GlooTransport()
    elif world > 1:
        obj = [_lib.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]

    c3 = args.workload == "c3"
    c5 = args.workload == "c5"
    c2 = args.workload == "c2"
    ts = args.workload == "c4ts"
    if args.size is None:
        args.size = 128 if (c3 or c2) else 256
    if args.ppc is None:
        args.ppc = 32 if (c3 or c2) else 43 if ts else 64
    S = args.size
    nd = 2 if c2 else 3
    if S % world:
        raise SystemExit("grid size must divide by the GPU count")
    if args.mg_graph is None:
        args.mg_graph = 1 if c2 else 0
    if args.mg_one_cu is None:
        args.mg_one_cu = 1 if c2 else 0
    cfg = configs.bench_config(args.workload, S, args.ppc, world, mg=args.mg, mg_shard=args.mg_shard,
                               mg_extrapolate=args.mg_extrapolate, mg_spectral_coarse=args.mg_spectral_coarse,
                               mg_graph=args.mg_graph, mg_one_cu=args.mg_one_cu,
                               obj_capacitance=args.obj_capacitance,
                               obj_second_guess=args.obj_second_guess, c5_fused=args.c5_fused, layout=args.layout,
                               sort_interval=args.sort_interval, sort_in_push=args.sort_in_push,
                               sort_fraction=args.sort_fraction, sort_max=args.sort_max,
                               sort_spread=args.sort_spread,
                               mg_smooth=args.mg_smooth if args.mg == "native" and args.mg_smooth != "ini" else None)
    nspecies = int(cfg["population"]["nSpecies"])
    # the one-workgroup solve applies (pinc_mg.c small_eligible): native, one
    # rank, 2-D, at most 16384 points
    one_cu = (args.mg == "native" and args.mg_one_cu == 1 and world == 1 and nd == 2 and S * S <= 16384
              and S & (S - 1) == 0)
    ini = configs.write_ini(cfg)
    spread_note = (f" and the blocks' mean cell box grew {args.sort_spread:g}x since the last sort"
                   if args.sort_spread > 0 else "")

    def barrier():
        if dist is not None:
            dist.barrier()

    def log(msg):
        print(f"[bench rank {rank}] {msg}", file=sys.stderr, flush=True)

    t_init0 = time.perf_counter()
    log(f"creating {S}^{nd} x {args.ppc} ppc on {world} GPU(s)")
    sim = Sim(ini, rank=rank, nranks=world, device=local, comm_id=comm_id, maxwell=not c2, perturb=c2,
              device_init=True, seed=20260101, timing=True, transport=transport)
    sim.init()
    sim.sync()
    t_init = time.perf_counter() - t_init0
    cycles_init = sim.cycles
    log(f"init {t_init:.1f} s, {sim.total_particles()} particles, {cycles_init} V-cycles")

    for i in range(args.warmup):
        tw = time.perf_counter()
        sim.step()
        sim.sync()
        log(f"warmup step {i}: {time.perf_counter() - tw:.2f} s, cycles {sim.cycles}")
    sim.timers_reset()
    c0 = sim.cycles
    _lib.probe_start("all", 4096)
    if world > 1:
        _lib.comm_stats_start(1 << 15)

    barrier()
    device_sync()
    sim.sync()
    t0 = time.perf_counter()
    # the steps run in the library in chunks of 10 (no return to Python
    # between steps; a progress line per chunk)
    done = 0
    chunk = 1 if os.environ.get("PINC_BENCH_PYLOOP") == "1" else 10  # (1: a Python call per step)
    while done < args.steps:
        k = min(chunk, args.steps - done)
        sim.step(k)
        done += k
        log(f"timed steps to {done} done at {time.perf_counter() - t0:.2f} s")
    sim.sync()
    device_sync()
    barrier()
    dt = time.perf_counter() - t0

    probes = {k: _lib.probe_read(k) for k in _lib.PROBES}
    phases = sim.timers()
    cycles = sim.cycles - c0
    n_local = sim.total_particles()
    ke, pe, _ = sim.energy()
    mg_levels = sim.mg_levels
    mg_halo = sim.mg_shard
    # particles that left through the slab faces in the last step (this
    # rank's; at one rank, those that would cross a slab boundary): the
    # migration exchange, one record of 2 nd + 1 doubles each
    em = sim.emigrants()   # [3^nd neighbours, species]
    slab_axis = (np.arange(3 ** nd) // 3 ** (nd - 1)) != 1
    z_emig = int(em[slab_axis].sum())

    dt_max = dt
    n_total = n_local
    comm = _lib.comm_stats_read() if world > 1 else {}
    rank_info = {"rank": rank, "wall_s": dt, "particles": n_local, "phase_ms": phases, "comm": comm,
                 "probes": {k: p for k, p in probes.items() if p["samples"] > 0}}
    all_info = [rank_info]
    if dist is not None:
        all_info = [None] * world
        dist.all_gather_object(all_info, rank_info)
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_max = float(t.item())
        c = torch.tensor([n_local], dtype=torch.int64, device=red_dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        n_total = int(c.item())

    K = args.steps
    value = n_total * K / dt_max
    ms_step = 1000.0 * dt_max / K
    solve_ms = phases["solve"] / K
    push_ms = (phases["move"] + phases["extract"] + phases["migrate"] + phases["deposit"] +
               phases["accelerate"]) / K
    kernels = {}
    ROCPROF_NAMES["spectral"] = "k_spectral_scale + rocFFT r2c/c2r kernels"
    ROCPROF_NAMES["push"] = "k_push<3, true, true, *>"
    if args.mg == "native":
        # two red-black iterations per launch (24 B per point: phi R+W, rho R)
        ROCPROF_NAMES["gs_pass"] = "k_gs_sweep4c<32, 8, 256>"
    sub = {}
    for k, p in probes.items():
        if p["samples"] == 0 or p["mean_ms"] <= 0:
            continue
        if k in _lib.SUB_PROBES:
            sub[k] = {"mean_launch_ms": p["mean_ms"], "launches": p["launches"], "samples": p["samples"],
                      "achieved_GBs": p["mean_bytes"] / (p["mean_ms"] * 1e-3) / 1e9}
            continue
        gbs = p["mean_bytes"] / (p["mean_ms"] * 1e-3) / 1e9
        rname = ROCPROF_NAMES[k]
        if k == "mg_cycle" and one_cu:
            rname = "k_mg_solve_small2<*> (every cycle of a solve and its convergence test, one launch)"
        elif nd == 2:
            rname = re.sub(r"<3,[^>]*>", "<2, *>", rname)
        kernels[k] = {"rocprof_name": rname, "mean_launch_ms": p["mean_ms"],
                      "bytes_per_launch": p["mean_bytes"], "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS,
                      "launches": p["launches"], "samples": p["samples"],
                      "est_ms_per_step": p["mean_ms"] * p["launches"] / args.steps}
    # the dominant kernel with algorithmic bytes (a replayed V-cycle graph,
    # "mg_cycle", is timed as a whole and has none: no roofline of its own)
    real = [k for k in kernels if kernels[k]["bytes_per_launch"] > 0] or list(kernels)
    dom = max(real, key=lambda k: kernels[k]["est_ms_per_step"])
    dk = kernels[dom]
    if "push_plain" in sub:
        for k in ("push_count", "push_sort"):
            if k in sub:
                sub[k]["vs_plain"] = sub[k]["mean_launch_ms"] / sub["push_plain"]["mean_launch_ms"]
    push_order = _push_order(_lib.probe_samples("push"))
    if push_order:
        sub["by_species"] = push_order
    # configuration key of the PMC traffic profiles (tools/pmc_summary.py)
    traffic_key = {"workload": args.workload, "grid": [S] * nd, "ppc_per_species": args.ppc, "n_gpus": world,
                   "layout": args.layout}

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "particle-updates/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (lattice positions, Maxwellian velocities from a seeded counter RNG)",
        "config": {
            "workload": (f"C2 Langmuir 2-D two-species plasma (input/langmuir2D.ini), {S}^2 grid, {args.ppc} ppc per "
                         f"species ({n_total} particles), 1D slab decomposition 1,{world}" if c2 else
                         ("C3 Maxwellian 3-D two-species plasma" if c3 else
                          f"C5 warm 3-D two-species plasma around an immersed sphere (radius {S / 32:g} cells)"
                          if c5 else "C4 two-stream variant: two electron beams (drift +-0.1 cells/step on every "
                          "component, population.c:385) and ions" if ts else "C4 warm 3-D two-species plasma")
                         + f", {S}^3 grid, {args.ppc} ppc per species "
                         f"({n_total} particles), 1D slab decomposition 1,1,{world}"),
            "grid": [S] * nd,
            "ppc_per_species": args.ppc,
            "species": nspecies,
            "particles": n_total,
            "decomposition": f"1,{world}" if c2 else f"1,1,{world}",
            "layout": args.layout + ((f" (per-species tile sort once {args.sort_fraction:g} of the particles left "
                                      f"their cell{spread_note}, at most {args.sort_max} steps apart)"
                                      if args.sort_fraction > 0 else
                                      f" (tile sort every {args.sort_interval} steps)") if args.layout == "tiled" else ""),
            "poisson": ("spectral (sSolver, rocFFT r2c/c2r, global grid)" if c3 else
                        (f"multigrid mgVRecursive, 2 levels used ({S}^{nd}, {S // 2}^{nd} solved exactly), "
                         if args.mg == "native" and args.mg_spectral_coarse else
                         f"multigrid mgVRecursive, {mg_levels} levels ({S}^{nd} down to {S >> (mg_levels - 1)}^{nd}), ")
                        + (f"RB Gauss-Seidel {cfg['multigrid']['nPreSmooth']}/{cfg['multigrid']['nPostSmooth']}/"
                           f"{cfg['multigrid']['nCoarseSolve']} (pre/post/coarse"
                           + ("; the reference ini's 10/10: --mg-smooth ini" if args.mg == "native" and
                              args.mg_smooth != "ini" else "") + "), ")
                        + ("native mode (correction scheme, coarse h^2 factor; the ini's 5 levels extended"
                           + (("; initial guesses extrapolated: the first solve of a step from the last two "
                               "steps' first solutions, the second from the first + "
                               + ("the exact discrete response to the correction charge (rocFFT)"
                                  if args.obj_second_guess == "spectral" else "the last correction response")
                               if c5 else "; initial guess 2 phi_n - phi_(n-1)") if args.mg_extrapolate else "")
                           + (("; two-grid: the level-1 correction solved exactly "
                               + ("in LDS through the real Fourier basis on the f64 matrix cores" if one_cu else
                                  "by rocFFT") + " with the 7-point symbol")
                              if args.mg_spectral_coarse else "")
                           + ("; every cycle of a solve and its convergence test in one workgroup "
                              "(multigrid:oneCU, k_mg_solve_small2)" if one_cu else "")
                           + "; RMS residual <= 1e-10 as the reference)"
                           if args.mg == "native" else "reference algorithm (parity mode)")
                        + (f", level 0 sharded over the slabs ({mg_halo} halo planes per side), levels >= 1 "
                           "all-gathered" if mg_halo else (", replicated on every rank" if world > 1 else ""))),
        },
        "poisson_ms_per_step": solve_ms,
        "push_deposit_ms_per_step": push_ms,
        "push_deposit_updates_per_s": n_local / (push_ms * 1e-3) * world if push_ms > 0 else None,
        "mg_cycles_per_solve": cycles / K,
        "phase_ms_per_step": {k: v / K for k, v in phases.items()},
        "init_s": t_init,
        "init_cycles": cycles_init,
        "migration": {"slab_face_emigrants_last_step": z_emig, "record_bytes": 8 * (2 * nd + 1),
                      "bytes_last_step": z_emig * 8 * (2 * nd + 1)},
        "energy": {"KE": ke, "PE": pe},
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "rocprof_name": dk["rocprof_name"],
            "achieved": dk["achieved_GBs"],
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": dk["frac"],
            "traffic": None,
            "traffic_note": "PMC HBM bytes per launch (FETCH_SIZE with the calibrated read correction + WRITE_SIZE, "
                            "MI355X_MICROARCH.md, profiles/*_pmc_calibration.json) from committed rocprofv3 passes "
                            "of this same configuration; null if none was profiled",
            "bytes_per_launch": dk["bytes_per_launch"],
            "mean_launch_ms": dk["mean_launch_ms"],
            "samples": dk["samples"],
            "launches": dk["launches"],
        },
        "kernels": kernels,
        "push_kinds": sub,
        "cpu_baseline": None,
    }
    if world > 1:
        result["multi_rank"] = _multi_rank_summary(all_info, K, dom, "host (gloo rehearsal, one GPU)"
                                                   if args.host_transport else "rccl")
    if not c3:
        # the smoothing counts the solve ran with, next to the reference ini's
        # (the native solve stops at the same 1e-10 RMS residual either way;
        # DESIGN.md section 6 has the 10/10 line measured beside the 4/4 one)
        result["config"]["mg_smooth"] = {"pre_post": [int(cfg["multigrid"]["nPreSmooth"]),
                                                      int(cfg["multigrid"]["nPostSmooth"])],
                                         "reference_ini": [10, 10]}
    result["config"]["traffic_key"] = traffic_key
    result["config"]["runtime_stack"] = _lib.runtime_stack()
    tr = _pmc_traffic(dk["rocprof_name"].rstrip("*").rstrip(" ,").split("*")[0], traffic_key)
    cc = _copy_ceiling_gbs()
    if cc and dom == "push":
        # the same achieved rate against what a pure copy of the push's own
        # streams reaches on this chip (a measured ceiling, not a spec)
        result["roofline"]["copy_ceiling"] = cc
        result["roofline"]["frac_of_copy_ceiling"] = dk["achieved_GBs"] / cc
        result["roofline"]["copy_ceiling_source"] = str(COPY_CEILING.relative_to(ROOT))
    if tr is not None:
        result["roofline"]["traffic"] = tr["bytes_per_launch"]
        result["roofline"]["traffic_source"] = tr["source"]
        result["roofline"]["traffic_ratio"] = tr["bytes_per_launch"] / dk["bytes_per_launch"]
    sim.close()
    os.unlink(ini)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_size, note = args.cpu_size, ""
        if cpu_size is None:
            # the full grid when the host holds the oracle's particles (AoS
            # pos+vel at the allocation, ~56 B per particle with buffers)
            need = 56.0 * (args.ppc + 8) * nspecies * S ** nd + 40.0 * 8 * S ** nd
            cpu_size = S if (c2 or _mem_available() > 1.3 * need) else 128
            if cpu_size != S:
                note = f" (the host's {_mem_available() / 2**30:.0f} GiB cannot hold the {S}^{nd} particles)"
        steps = args.cpu_steps if args.cpu_steps is not None else (3 if cpu_size >= 256 else 20)
        result["cpu_baseline"] = _cpu_baseline(cpu_size, args.ppc, steps,
                                               args.mg == "native", args.workload if args.workload != "c5" else "c4",
                                               # the oracle's exact coarse solve is a naive DFT (no FFT
                                               # library here): the CPU keeps the V-cycle below level 1,
                                               # which converges in as many cycles and is faster there
                                               args.mg_extrapolate, 0, note)
    if rank == 0:
        print(json.dumps(result), file=out, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
