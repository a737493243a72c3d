"""Benchmark: RK45 ray-steps/s of the MI355X ray integrator (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--days D] [--bg zonal|nonzonal]

One "step" = one pass of the hot path over ONE ray set: the whole C3 workload
(2-degree global seed grid x k = 1..10 x periods {inf, 50, 30, 20, 10} d =
2.40 M ray slots, of which 0.72 M have a real initial root) integrated for 90
days (1081 output rows at 2 h) -- GPU initial rows, solver construction, the
ray loop and every output row included.  Inputs are resident in HBM when the
timed region starts.

With N ranks (one per GPU; BASELINE configs[3] = C4; `--gpus N` starts them,
or torch.distributed.run does) the SAME set is split across the GPUs
(shard.run_sharded, scaling "strong", the default):
inside each timed step rank 0's basic state is broadcast over RCCL, every rank
builds the initial rows and runs a 6-row probe launch over every ray, the
probe's per-ray attempts decide a cost-balanced split (no communication: the
same deterministic rule on every rank), each rank integrates its own rays to
90 days, and the last row and step counters of every ray are gathered to
rank 0 over RCCL.  value = the set's accepted ray-steps / the slowest rank's
wall time.  ``--scaling weak`` (every rank its own C3 set) is a diagnostic:
its aggregate is reported under ``weak_scaling``, never as ``value``.

Rank 0 prints ONE JSON line.  ``roofline`` prices the ray-loop kernel at the
bound it actually hits -- VALU instruction issue at one wave per SIMD (PMC
SQ_INSTS_VALU x 4 cycles against 1024 SIMDs x the in-kernel clock) -- with the
real HBM traffic (PMC) and the algorithmic 2112 B per ray-step of SURVEY.md
§8(d) beside it; ``cpu_baseline`` times the NumPy oracle (oracle/rwrt_oracle.py,
bit-exact with the reference) on a bounded sample of the same rays on the host.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rossby-wave-ray-tracing_amd"))

import torch  # noqa: E402

import synthetic as S  # noqa: E402

METRIC = "ray-steps/sec (whole node), 10^6 rays RKF45; max |Δpos| vs CPU ref"
BYTES_PER_STEP = 2112          # 6 RHS evals x 4 corners x 11 fields x 8 B
HBM_PEAK = 8.0e12              # MI355X_MICROARCH.md, chip-level parameters
FLOP_PER_STEP = 2.0e3          # fp64 FLOP per accepted ray-step (~1462 per attempt x 1.39)
FP64_PEAK = 78.6e12            # MI355X vector FP64 (16 lanes x FMA per SIMD-cycle x 1024 SIMDs x 2.4 GHz)


def c3_rows(bs, lon_offset_deg=0.0, periods=S.C3_PERIODS_DAYS):
    """The 7 initial rows (lon lat k l amp ug vg; ``WR.ray_initial_numpy``,
    host) of every C3 slot, all periods concatenated: ``[7, nslot]``."""
    from wr import initial_rows
    cfg = S.config("C3")
    deg2rad = np.pi / 180.0
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    lon = (((cfg.SW_lon + lon_offset_deg) % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * deg2rad
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * deg2rad
    ys = []
    for P in periods:
        with np.errstate(all="ignore"):
            rows = initial_rows(bs, lon, lat, cfg.zwn, S.c3_freq(P))
        ys.append(np.array(rows).reshape(7, -1))
    return np.concatenate(ys, axis=1)


def c3_initial_state(bs, lon_offset_deg=0.0, periods=S.C3_PERIODS_DAYS):
    """Initial ray state y0[5, nslot] of C3 (all periods concatenated)."""
    return np.ascontiguousarray(c3_rows(bs, lon_offset_deg, periods)[:5])


def c3_sources(eng, lon_offset_deg=0.0, periods=S.C3_PERIODS_DAYS):
    """Device inputs of the GPU initialiser for C3: the source list and one
    per-k constant block per period."""
    cfg = S.config("C3")
    deg2rad = np.pi / 180.0
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    lon = (((cfg.SW_lon + lon_offset_deg) % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * deg2rad
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * deg2rad
    return eng.sources(lon, lat), [eng.zwn_tensor(cfg.zwn, S.c3_freq(P)) for P in periods]


def make_bs(kind="zonal"):
    from bs import BS
    bg = S.background(kind)
    bs = BS(len(bg["lon"]), len(bg["lat"]))
    bs.load_arrays(**bg)
    bs.ready(xcyclic=True)
    return bs, bg


def cpu_baseline(bg, y0, nrays, days, seed=0, fsal=True, pick=None):
    """Time the oracle on ``nrays`` live rays for ``days`` (1 host core) --
    a random sample, or the rays ``pick``.  ``fsal=False``: the reference's
    loop shape (f recomputed for every column at each step start,
    rkf45.py:378).  Returns (pick, hist, accepted, seconds, nt, rejected, RHS
    columns evaluated)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rwrt_oracle as O
    if pick is None:
        rng = np.random.default_rng(seed)
        live = np.where(~np.isnan(y0.mean(axis=0)))[0]
        pick = np.sort(rng.choice(live, size=min(nrays, len(live)), replace=False))
    ob = O.Background(**bg)
    nt = int(round(days * 12)) + 1
    cols = [0]
    t0 = time.perf_counter()
    with np.errstate(all="ignore"):
        hist, nacc, nrej, st = O.ray_run(ob, y0[:, pick].copy(), nt, 7200.0, fsal=fsal, columns=cols)
    dt = time.perf_counter() - t0
    return pick, hist, int(nacc.sum()), dt, nt, int(nrej.sum()), cols[0]


def cpu_baseline_mp(bg, y0, procs, rays_per_proc, days, seed=1):
    """The oracle on ``procs`` host processes (rays are independent), each on
    its own ``rays_per_proc`` live C3 rays for ``days``; rate = all accepted
    steps / the slowest process's ray-loop time."""
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rwrt_oracle as O
    rng = np.random.default_rng(seed)
    live = np.where(~np.isnan(y0.mean(axis=0)))[0]
    pick = rng.choice(live, size=min(procs * rays_per_proc, len(live)), replace=False)
    nt = int(round(days * 12)) + 1
    jobs = [(bg, y0[:, part].copy(), nt, 7200.0, False) for part in np.array_split(pick, procs)]
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(O.ray_run_timed, jobs)
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return steps, wall, len(pick)


def library_sha():
    """sha256 (16 hex digits) of the librwrt.so this process loaded: a
    profile summary counts for this run only if it was taken on the same build."""
    import hashlib
    import _hip as H
    return hashlib.sha256(open(H.LIB_PATH, "rb").read()).hexdigest()[:16]


def endpoint_sha(ends):
    """sha256 (16 hex digits) of a ray set's last rows (NaN canonicalised):
    rank 0's set is the same at every N (weak scaling), so its endpoints must
    hash the same in the 1-GPU and the N-GPU lines."""
    import hashlib
    e = ends.detach().cpu().numpy().astype(np.float64, copy=True)
    e[np.isnan(e)] = np.nan
    return hashlib.sha256(np.ascontiguousarray(e).tobytes()).hexdigest()[:16]


def find_profile(name, path, workload, schedule):
    """A per-launch profile summary (profiles/<round>/.../<name>) of this
    workload run with the same launch schedule (rows per launch), taken on
    this build of the library if one is committed (else the newest, flagged)."""
    import glob
    # newest profile first by path (profiles/<round>/<version>/...: sorts the
    # same in any checkout, unlike file times)
    cands = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "**", name), recursive=True),
                                       reverse=True)
    sha, fallback = library_sha(), (None, None)
    for c in cands:
        try:
            t = json.load(open(c))
        except (OSError, ValueError):
            continue
        if t.get("workload") == workload and t.get("launch_rows") == schedule:
            if t.get("library_sha256") == sha:
                return t, os.path.relpath(c, ROOT)
            if fallback[0] is None:
                fallback = (dict(t, profile_of_other_build=True), os.path.relpath(c, ROOT))
    return fallback


def roofline(steps_per_launch, avg_launch_s, workload, schedule, bytes_per_step, args, bound="valu_issue",
             steps_per_s_gpu=None):
    """The ray-loop kernel against the bound it hits: VALU issue at one wave per
    SIMD.  VALU wave-instructions per launch and the in-kernel clock come from
    the PMC profile of this build and schedule (tools/pmc_valu.py), the launch
    time from this run's HIP events.  Real HBM bytes (PMC) and the algorithmic
    bytes of SURVEY.md §8(d) are reported beside it."""
    valu, vsrc = find_profile("valu.json", args.valu_profile, workload, schedule)
    traffic, tsrc = find_profile("traffic.json", args.traffic, workload, schedule)
    alg = steps_per_launch * bytes_per_step / avg_launch_s
    out = {"bound": "valu_issue", "achieved": None, "peak": None, "unit": "G VALU wave-instructions/s",
           "frac": None, "traffic": traffic["traffic_bytes_per_launch"] if traffic else None,
           "kernel": "rk45_run_kernel", "avg_launch_ms": 1e3 * avg_launch_s,
           "valu_source": vsrc, "traffic_source": tsrc,
           "profile_same_build": bool(valu) and not valu.get("profile_of_other_build", False)}
    if valu:
        ach = valu["valu_insts_per_launch"] / avg_launch_s
        peak = valu["simds"] * valu["clock_hz"] / valu["cycles_per_valu"]
        out.update(achieved=ach / 1e9, peak=peak / 1e9, frac=ach / peak,
                   valu_insts_per_launch=valu["valu_insts_per_launch"],
                   clock_GHz=valu["clock_hz"] / 1e9,
                   valu_peak_basis=("4 cycles per wave64 VALU instruction: the SIMD's fp64 rate (16 lanes "
                                    "per cycle, the 78.6 TF vector FP64 peak) and the one-wave-per-SIMD "
                                    "issue ceiling of this kernel (256 VGPR + AGPRs, 146 KB LDS per block). "
                                    "32-bit VALU work issues in 2 cycles when a second wave shares the "
                                    "SIMD (MI355X_MICROARCH.md:54,473), so against the chip's mixed-width "
                                    "ceiling this frac is an upper bound"),
                   note=("one wave per SIMD (256 VGPR + AGPRs, 146 KB LDS per block): every VALU "
                         "wave-instruction holds its SIMD's issue for >= 4 cycles; peak = 1024 SIMDs x "
                         "in-kernel clock (GRBM_GUI_ACTIVE / 8 / kernel time) / 4"))
        if "issue_active_frac" in valu:
            # any instruction type (VALU, SALU, LDS, VMEM, branch) takes the wave's
            # issue slot at one wave per SIMD: the share of wave cycles that issued
            out["issue_any"] = {"frac_of_wave_cycles": valu["issue_active_frac"],
                                "valu_frac_of_wave_cycles": valu.get("valu_active_frac"),
                                "counters": "SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES"}
    out["hbm"] = {"achieved_GBps": traffic["traffic_bytes_per_launch"] / avg_launch_s / 1e9 if traffic else None,
                  "peak_GBps": HBM_PEAK / 1e9,
                  "frac": traffic["traffic_bytes_per_launch"] / avg_launch_s / HBM_PEAK if traffic else None,
                  "unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)"}
    out["algorithmic"] = {"bytes_per_ray_step": bytes_per_step, "GBps": alg / 1e9,
                          "frac_of_hbm_peak": alg / HBM_PEAK,
                          "bound": ("none: not an HBM bound (the lookups it counts are served by the LDS "
                                    "cell cache and L2; >= 1 by construction at 2.5 degrees)"
                                    if alg >= HBM_PEAK else
                                    "a yardstick: the measured line traffic (hbm) is the HBM figure"),
                          "note": ("SURVEY.md 8(d): 6 RHS x 4 corners x 11 fields x 8 B per accepted step; "
                                   "most lookups are served by the per-lane LDS cell cache and L2, so this "
                                   "is a yardstick, not HBM traffic, and can exceed the HBM peak")}
    if steps_per_s_gpu is not None:
        # the arithmetic the path needs, against the vector FP64 peak
        out["fp64_flop_frac"] = steps_per_s_gpu * FLOP_PER_STEP / FP64_PEAK
        out["fp64_flop"] = {"flop_per_ray_step": FLOP_PER_STEP, "TFLOPs": steps_per_s_gpu * FLOP_PER_STEP / 1e12,
                            "peak_TFLOPs": FP64_PEAK / 1e12,
                            "note": "SURVEY.md 8(d): ~1462 fp64 FLOP per DP5(4) attempt x 1.39 attempts per "
                                    "accepted step, transcendentals excluded; per GPU"}
    if bound == "hbm":
        # C5: the 0.25-degree levels are gathered from HBM / MALL (one level per
        # lane cached in LDS): the memory roofline leads, VALU issue beside it
        valu_part = {k: out[k] for k in ("achieved", "peak", "unit", "frac", "note") if k in out}
        out.update(bound="hbm", unit="GB/s", peak=HBM_PEAK / 1e9, achieved=out["hbm"]["achieved_GBps"],
                   frac=out["hbm"]["frac"], valu_issue=valu_part,
                   note=("PMC line traffic (FETCH_SIZE x2 + WRITE_SIZE, calibrated on this access pattern: "
                         "DESIGN.md 4, C5 traffic) per launch over the launch's HIP-event time"))
    return out


def _split_arg(s):
    """--split: 'off', 'auto' or 'auto:a,b,..' (positive row counts)"""
    import argparse
    head, colon, rows = s.partition(":")
    if s in ("off", "auto") or (head == "auto" and colon and all(x.isdigit() and int(x) > 0
                                                                  for x in rows.split(","))):
        return s
    raise argparse.ArgumentTypeError(f"--split: 'off', 'auto' or 'auto:a,b,..', not {s!r}")


def schedule_defaults(args, world):
    """The schedule knobs left unset on the command line, by what one GPU
    holds: a whole C3 set (one GPU, or weak scaling) or a split one / C5.
      first launches  24 + 160 rows (a whole set: throughput-bound, a longer
                      second re-ordering launch orders the last one better,
                      profiles/r2/ab/launch_sweep.txt); a split C3 set 96
                      (chain-bound ranks: one re-ordering launch fewer, 8
                      ranks 0.196 s against 0.201 with 24 + 96, 24 alone
                      0.259 -- profiles/r6/c4_lead_sweep.txt); C5 24 + 96;
      probe           4 rows for a whole C3 set (+0.75 % over 6 with the
                      per-launch latency mode, profiles/r3/sched/pass_w_*),
                      6 otherwise;
      latency mode    a whole zonal C3 set: the 64 heaviest rays of each
                      launch after the probe (one latency-mode block: the
                      launches are bound by their heaviest rays' chains; 64 /
                      64 / 64 measured +0.4 % over round 3's 64 / 256 / 64 and
                      +1.3 % over none, profiles/r4/sched/team.txt -- more
                      latency-mode blocks make each attempt slower, DESIGN.md
                      §4); a whole non-zonal set: none (its chain-bound rays
                      are not the predicted heaviest; 64/256/64 costs 1.5 %,
                      pass_x_*); a split set: the auto rule (RayEngine.team_size)."""
    whole = args.config == "C3" and (world == 1 or args.scaling == "weak")
    if args.first_chunk is None:
        args.first_chunk = "24,160" if whole else ("96" if args.config == "C3" else "24,96")
    if args.probe is None:
        args.probe = 4 if whole else 6
    if args.team is None:
        # (C5: none -- the rays that end a split C5 launch are not the heaviest
        # of the launches before it, profiles/r5/c5lat/)
        args.team = ("64,64,64" if args.bg == "zonal" else "0") if whole else ("0" if args.config == "C5" else "auto")
    return args


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def resolve_world(gpus, env=None):
    """How this process takes part in an N-GPU run: ``("spawn", N)`` -- no
    launcher set WORLD_SIZE and N > 1, so this process starts the N ranks
    itself -- or ``("rank", world)`` -- run as one rank (N = 1, or under
    torch.distributed.run).  ``--gpus`` that disagrees with a launcher's
    WORLD_SIZE is an error, never silently ignored."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        return "rank", world
    n = 1 if gpus is None else int(gpus)
    if n < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {n})")
    return ("spawn", n) if n > 1 else ("rank", 1)


def spawn_ranks(n, argv, timeout=None):
    """Start ``n`` ranks of this script (one per GPU, local rank r -> GPU r),
    rendezvous on 127.0.0.1; rank 0 prints the JSON line.  The parent never
    touches the GPU (it only starts children and waits), and a rank that fails
    takes the others down with it.  Returns the worst exit code."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    t0 = time.time()
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        late = timeout is not None and time.time() - t0 > timeout
        if bad or late:
            rc = bad[0] if bad else 124
            for p in procs:
                if p.poll() is None:
                    p.send_signal(signal.SIGTERM)
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    for p in procs:
        rc = rc or (p.returncode or 0)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each); without a launcher, N > 1 starts the N ranks itself")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong (default; BASELINE configs[3]): ONE C3 set split over the ranks by "
                         "measured cost (shard.run_sharded).  weak (diagnostic, not a BASELINE config): "
                         "every rank integrates its own full C3 set (the seed grid shifted by rank x 2/N "
                         "degrees of longitude) -- reported under 'weak_scaling', never as 'value'")
    ap.add_argument("--dry-run", action="store_true",
                    help="set up the ranks and the process group, print the line's skeleton, stop "
                         "(tests the launcher without a GPU)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--days", type=float, default=90.0, help="integration horizon per step")
    ap.add_argument("--chunk", type=int, default=0, help="output rows per kernel launch")
    ap.add_argument("--cpu-rays", type=int, default=16384)
    ap.add_argument("--cpu-days", type=float, default=12.0)   # ~10 s of 1-core oracle work
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="processes of the multi-core CPU baseline (1: skip it)")
    ap.add_argument("--periods", type=int, default=5, help="C3 periods in the batch (1-5)")
    ap.add_argument("--bg", default="zonal", choices=["zonal", "nonzonal"],
                    help="C3 basic state: the DJF jets (SURVEY.md 8(d)) or their non-zonal variant")
    ap.add_argument("--order", default=None, choices=["priority", "cost", "cell", "total", "live"],
                    help="work-queue order: longest-first by the previous launch's work (priority, "
                         "cost; C3's default), cost classes then Morton order of the rays' cells (cell; "
                         "C5's default: its lookups are HBM gathers), by all work so far (total), or "
                         "live-first")
    ap.add_argument("--probe", type=int, default=None,
                    help="rows of the probe launch over every ray whose attempts split and order the set "
                         "(default: 4 for a whole C3 set per GPU, 6 otherwise)")
    ap.add_argument("--first-chunk", default=None,
                    help="rows of the short launches after the probe that re-measure per-ray cost "
                         "(default: C3 on one GPU 24,160 -- profiles/r2/ab/launch_sweep.txt --, "
                         "otherwise 24,96)")
    ap.add_argument("--config", default="C3", choices=["C3", "C5"],
                    help="C3 (BASELINE configs[2]/[3], the metric's workload) or C5 (configs[4]: "
                         "0.25-degree time-varying background)")
    ap.add_argument("--fields", default="fp64", choices=["fp64", "fp32", "fp32a"],
                    help="C5: storage of the background levels (fp64 arithmetic), or fp32a: fp32 "
                         "levels and an fp32 RHS (fp64 positions, time and stepper)")
    ap.add_argument("--c5-periods", type=int, default=5,
                    help="C5 periods (1-5 of the C3 list; 5 = 9.67 M slots, ~4 M live rays: BASELINE's size)")
    ap.add_argument("--split", default="auto", type=_split_arg,
                    help="'auto': split the long launch once more when the leading launches' per-ray "
                         "work predicts the next poorly (RayEngine.SPLIT_RHO), after SPLIT_ROWS rows; "
                         "'auto:a,b,..': cut after a, a+b, .. rows instead; 'off'")
    ap.add_argument("--team", default=None,
                    help="rays per launch in latency mode (quad_rays: four lanes of a wave per ray); "
                         "an integer, one per launch after the probe (e.g. 64,256,64; the last "
                         "repeats) or 'auto' (RayEngine.team_size).  Default: 64,64,64 for a whole C3 "
                         "set per GPU, auto for a split one")
    ap.add_argument("--shard-probe", type=int, default=1, choices=[0, 1],
                    help="N > 1 (strong): each rank probes 1/N of the rays and the probe costs are "
                         "all-gathered (shard.probe_costs; 0: every rank probes every ray)")
    ap.add_argument("--lib", default=None, help="alternative librwrt build (A/B timing)")
    ap.add_argument("--traffic", default=None, help="traffic.json (tools/pmc_traffic.py)")
    ap.add_argument("--valu-profile", default=None, help="valu.json (tools/pmc_valu.py)")
    ap.add_argument("--replicate", type=int, default=1,
                    help="diagnostic: repeat the ray batch k times (more rays per lane)")
    args = ap.parse_args()
    if args.order is None:
        args.order = "cell" if args.config == "C5" else "priority"
    how, world = resolve_world(args.gpus)
    if how == "spawn":
        # no launcher: start the N ranks here, before anything touches the GPU
        return spawn_ranks(world, sys.argv[1:])
    schedule_defaults(args, world)
    if args.lib:
        os.environ["RWRT_LIB"] = os.path.abspath(args.lib)

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = group = None
    backend = None
    share = 1                                    # ranks sharing this rank's GPU
    if world > 1:
        import torch.distributed as dist
        # one GPU per rank over RCCL ("nccl"); with fewer GPUs than ranks (the
        # one-GPU rehearsal) ranks share a device and talk over gloo
        ndev = torch.cuda.device_count()
        share = max(1, -(-world // max(ndev, 1)))
        backend = os.environ.get("RWRT_DIST_BACKEND") or ("nccl" if ndev >= world else "gloo")
        if ndev:
            local = local % ndev
            torch.cuda.set_device(local)
        dist.init_process_group(backend, rank=rank, world_size=world)
        group = dist.group.WORLD
    if args.dry_run:
        if dist:
            t = torch.ones(1)
            if backend == "gloo":
                dist.all_reduce(t)
            dist.barrier()
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "dry_run": True,
                              "backend": backend, "scaling": args.scaling,
                              "world_sum": float(t.item()) if dist else 1.0}), flush=True)
        if dist:
            dist.destroy_process_group()
        return 0
    dev = torch.device("cuda", local if world > 1 else 0)

    if args.config == "C5":
        return main_c5(args, dist, group, rank, world, dev, share)
    from engine import RayEngine
    from shard import broadcast_array, run_sharded
    weak = args.scaling == "weak"
    bs, bg = make_bs(args.bg)
    periods = S.C3_PERIODS_DAYS[: args.periods]
    # weak scaling: rank r traces the C3 seed grid shifted by r x dlon / N
    # degrees of longitude (N GPUs: an N-times denser grid; rank 0 = C3)
    offset = rank * S.config("C3").dlon / world if weak else 0.0
    t_init = time.perf_counter()
    y0 = c3_initial_state(bs, offset, periods=periods) if (rank == 0 or args.replicate > 1) else None
    t_init = time.perf_counter() - t_init
    if args.replicate > 1:
        y0 = np.concatenate([y0] * args.replicate, axis=1)
    # the basic state every rank integrates through is rank 0's (bs.py:202-262
    # reads its file on one process): its field stack broadcast before the
    # timed steps, then rank 0's packed state again inside every step
    fields = broadcast_array(bs.fields if rank == 0 else None, group=group) if dist else bs.fields
    eng = RayEngine(fields, bs.lon, bs.lat, device=dev)
    nt = int(round(args.days * 12)) + 1
    gpu_init = args.replicate == 1
    init_same = None
    if gpu_init:
        # sources and per-k constants resident in HBM; the step starts from them
        src, zcs = c3_sources(eng, offset, periods)
        init_rows = [None] * len(zcs)
        init_info = torch.zeros(1, dtype=torch.int32, device=dev)

        def make_y0():
            ys = []
            for j, zc in enumerate(zcs):
                init_rows[j], _ = eng.initial_rows_dev(src, zc, init_rows[j], init_info)
                ys.append(init_rows[j][:5].reshape(5, -1))
            return torch.cat(ys, dim=1)
        y0_d = make_y0()
        if y0 is not None:
            hy = torch.as_tensor(y0)
            init_same = bool(((y0_d.cpu() == hy) | (torch.isnan(y0_d.cpu()) & torch.isnan(hy))).all())
    else:
        y0_d = torch.as_tensor(y0, device=dev)
    nslot = y0_d.shape[1]
    live_idx = torch.nonzero(~torch.isnan(y0_d.sum(0))).squeeze(1)
    n_live = int(live_idx.numel())
    # this rank's rows stay in HBM (C3 on one GPU: 166 GB of 288 GB), so the
    # ray loop is a few launches: the probe, two short re-ordering launches,
    # then all the rest (ranks sharing a GPU share its memory)
    # row blocks for the live rays only (rwrt_rk45_run_slots, ABI 4): this
    # rank's live rays bound them (cost_partition deals the live rays snake-wise)
    n_blk = n_live if weak else -(-n_live // world) + 2
    free = torch.cuda.mem_get_info(dev)[0] // share
    chunk = args.chunk or max(1, min(nt - 1, int(0.8 * free) // (max(n_blk, 1) * 64)))
    out = torch.empty((max(n_blk, 1), min(chunk, nt - 1), 8), dtype=torch.float64, device=dev)
    lead = [int(x) for x in str(args.first_chunk).split(",") if x]
    team = (args.team if args.team == "auto" else
            [x if x == "auto" else int(x) for x in args.team.split(",")] if "," in args.team else int(args.team))
    split = None if args.split == "off" else args.split
    gather_dev = torch.device("cpu") if backend == "gloo" else dev
    n_live_max = n_live
    if weak and dist:
        t = torch.tensor([n_live], dtype=torch.int64, device=gather_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        n_live_max = int(t.item())
    gathered = {}

    def gather_endpoints(r):
        """Weak scaling: every rank's live rays' last rows (lon lat k l amp ug
        vg nacc) gathered to rank 0 (RCCL gather over xGMI)."""
        ends = r.endpoints[live_idx]
        if not dist:
            gathered["rank0"] = ends
            return
        pad = torch.full((n_live_max, 8), float("nan"), dtype=torch.float64, device=gather_dev)
        pad[:n_live] = ends.to(gather_dev)
        bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
        dist.gather(pad, bufs, dst=0, group=group)
        if rank == 0:
            gathered["rank0"] = bufs[0][:n_live]
            gathered["all"] = bufs

    def one_step(events=None):
        if dist is not None:
            dist.broadcast(eng.packed, 0, group=group)   # rank 0's basic state (RCCL over xGMI)
        y = make_y0() if gpu_init else y0_d
        if weak:
            r = run_sharded(eng, y, nt, 7200.0, rank=0, world=1, probe=args.probe, lead=lead,
                            chunk=chunk, out=out, events=events, ttotal=(nt - 1) * 7200.0,
                            order_policy=args.order, team=team, split=split)
            gather_endpoints(r)
            return r
        return run_sharded(eng, y, nt, 7200.0, group=group, probe=args.probe, lead=lead,
                           chunk=chunk, out=out, events=events, ttotal=(nt - 1) * 7200.0,
                           order_policy=args.order, team=team, split=split, shard_probe=bool(args.shard_probe))

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    events, steps_done = [], 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = one_step(events)
        steps_done += r.steps_local
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rows_bytes = int(eng.rows_bytes)   # (the timed steps' row buffers; later sample runs reuse the engine)
    kern_s = sum(a.elapsed_time(b) for a, b in events) / 1e3
    rej = int(r.res.nrej.sum().item())
    n_mine = int(r.idx.numel())

    tot_steps, max_el, tot_rej = steps_done, elapsed, rej
    if dist:
        t = torch.tensor([float(steps_done), elapsed, float(rej)], dtype=torch.float64, device=gather_dev)
        s = t.clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        m = t.clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot_steps, max_el, tot_rej = s[0].item(), m[1].item(), s[2].item()

    result = None
    if rank == 0:
        value = tot_steps / max_el
        per_launch_steps = steps_done / max(len(events), 1)
        avg_launch_s = kern_s / max(len(events), 1)
        workload = (f"C3: 2deg global seeds x k=1..10 x {args.periods} periods, "
                    f"{args.days:g} d at 2 h, 2.5deg DJF jet background"
                    + (" (non-zonal variant)" if args.bg == "nonzonal" else "")
                    + (" (BASELINE configs[2])" if world == 1 else
                       (" per GPU, the seed grid shifted by rank x 2/N deg of longitude (BASELINE configs[3], "
                        "weak scaling)" if weak else " (BASELINE configs[3]: C4, one set split)")))
        schedule = [args.probe] + [b - a for a, b in r.res.bounds]
        if weak:
            par = (f"{world} rank(s), one GPU each (backend {backend or 'none'}): each integrates its own "
                   f"C3 seed grid (2.40 M slots), no exchange during integration; inside the timed step "
                   f"rank 0's basic state is broadcast (RCCL) and every rank's live-ray endpoints + "
                   f"accepted-step counts are gathered to rank 0 (RCCL gather)")
        else:
            par = (f"one ray set over {world} GPU(s): cost-balanced split by a "
                   f"{args.probe}-row probe" +
                   (" (each rank probes 1/N of the rays, the costs all-gathered)" if world > 1 and args.shard_probe
                    else "") +
                   ", RCCL broadcast of the basic state and gather of endpoints + step counters inside the "
                   "timed step")
        ends0 = gathered.get("rank0") if weak else r.endpoints[live_idx.to(r.endpoints.device)]
        result = {
            "metric": METRIC, "value": value, "unit": "ray-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * max_el / args.steps, "higher_is_better": True,
            "scaling": "weak" if weak else "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload,
                       "ray_slots": nslot * (world if weak else 1), "live_rays_rank0": n_live,
                       "rows": nt, "rows_per_launch": chunk, "launch_rows": schedule,
                       "rank0_rays": n_mine,
                       "latency_mode": ("per launch, the heaviest rays whose move to quad_rays (four lanes of a "
                                        "wave per ray) minimises the predicted makespan by >= 10 %"
                                        if args.team == "auto"
                                        else f"{args.team} heaviest rays per launch after the probe in "
                                             f"latency mode (quad_rays, four lanes of a wave per ray)"),
                       "parallelism": par},
            "ray_steps_per_step": tot_steps / args.steps,
            "ray_steps_per_step_rank0": steps_done / args.steps,
            "rows_bytes": {"rank0": rows_bytes,
                           "dense_equivalent": int(r.idx.numel()) * min(chunk, nt - 1) * 64,
                           "note": "rank 0's device row buffer: row blocks for the rays live at a launch's "
                                   "start only (rwrt_rk45_run_slots); frozen rays' rows are tails"},
            "rejected_per_accepted": tot_rej * args.steps / max(tot_steps, 1),
            "host_init_s": t_init,
            "init": ("GPU rwrt_ray_initial inside every timed step (bit-identical to the host rows)"
                     if gpu_init else "host NumPy rows, outside the timed region"),
            "init_bitwise_vs_host": init_same,
            "endpoints_rank0_sha256": endpoint_sha(ends0) if ends0 is not None else None,
            "queue_order": args.order,
            "long_launch_split": {"mode": args.split, "rank_corr_of_leading_launches": eng.split_rho,
                                  "threshold": eng.SPLIT_RHO, "rows": eng.SPLIT_ROWS},
            "library": os.path.basename(os.environ.get("RWRT_LIB", "librwrt.so")),
            "library_sha256": library_sha(),
            "roofline": roofline(per_launch_steps, avg_launch_s, workload, schedule, BYTES_PER_STEP, args,
                                 steps_per_s_gpu=value / world),
        }
        if weak and "all" in gathered:
            result["gathered_endpoints"] = {
                "rows_per_rank": n_live_max, "bytes": world * n_live_max * 64,
                "alive_at_end": int(sum(int((~torch.isnan(b[:, 0])).sum().item()) for b in gathered["all"]))}
        if world == 1 and not args.no_cpu:
            pick, hist, csteps, cdt, cnt, crej, ccols = cpu_baseline(bg, y0, args.cpu_rays, args.cpu_days)
            # the reference's own loop shape, timed on the first half of the
            # same sample (~2x the RHS work per step)
            rpick, _, rsteps, rdt, _, _, rcols = cpu_baseline(bg, y0, args.cpu_rays // 2, args.cpu_days,
                                                               fsal=False, pick=pick[: len(pick) // 2])
            result["cpu_baseline"] = {
                "value": rsteps / rdt, "unit": "ray-steps/s", "cores": 1, "kind": "reference_loop",
                "sample": f"{len(rpick)} live C3 rays x {args.cpu_days:g} d ({rsteps} ray-steps, {rdt:.1f} s) "
                          f"with oracle/rwrt_oracle.py in the reference's loop shape: f = fun(t, y) "
                          f"recomputed for every column at each step start (rkf45.py:378) and the rejected "
                          f"subsets re-run (rkf45.py:410-502) -- {rcols / max(rsteps, 1):.1f} RHS columns per "
                          f"accepted step; the reference's arithmetic bit for bit (NumPy)",
                "rhs_columns_per_accepted_step": rcols / max(rsteps, 1),
                "survey_reference_rate_per_core": "5-6e4 ray-steps/s (BASELINE.md; SURVEY.md 8(d), the "
                                                  "reference itself on the survey host)",
                "port_fsal": {"value": csteps / cdt, "unit": "ray-steps/s", "cores": 1, "kind": "port",
                              "sample": f"{len(pick)} live C3 rays x {args.cpu_days:g} d ({csteps} ray-steps, "
                                        f"{cdt:.1f} s), FSAL: {ccols / max(csteps, 1):.1f} RHS columns per "
                                        f"accepted step"},
                "host_cpus": os.cpu_count()}
            if args.cpu_procs > 1:
                msteps, mwall, mrays = cpu_baseline_mp(bg, y0, args.cpu_procs, args.cpu_rays // 8,
                                                       args.cpu_days)
                result["cpu_baseline_mp"] = {
                    "value": msteps / mwall, "unit": "ray-steps/s", "cores": args.cpu_procs,
                    "kind": "reference_loop",
                    "sample": f"{mrays} live C3 rays x {args.cpu_days:g} d over {args.cpu_procs} "
                              f"processes in the reference's loop shape ({msteps} ray-steps, slowest "
                              f"process {mwall:.1f} s)"}
            # parity of the same sample on the GPU after the same horizon
            rows = {}
            eng.integrate(torch.as_tensor(y0[:, pick], device=dev), cnt, 7200.0,
                          sink=lambda a, b, o: rows.__setitem__(a, o[:, :, :7].cpu().numpy()))
            gpu = np.concatenate([rows[k] for k in sorted(rows)], axis=1)   # rows 1..cnt-1
            parity = []
            for row in sorted({1, min(12, cnt - 1), min(48, cnt - 1), cnt - 1}):
                g, c = gpu[:, row - 1, :2], hist[:2, row].T
                ok = ~np.isnan(g).any(1) & ~np.isnan(c).any(1)
                d = np.max(np.abs(g[ok] - c[ok]), axis=1) if ok.any() else np.zeros(1)
                parity.append({"horizon_days": row / 12.0, "rays": int(ok.sum()),
                               "p50": float(np.median(d)), "p99": float(np.percentile(d, 99)),
                               "max": float(d.max()), "frac_gt_1e-6": float(np.mean(d > 1e-6)),
                               "alive_mismatch": int(np.sum(np.isnan(g[:, 0]) != np.isnan(c[:, 0])))})
            result["max_dpos_vs_cpu_rad"] = parity
            g7, c7 = np.transpose(gpu, (2, 1, 0)), hist[:, 1:]
            same = (g7 == c7) | (np.isnan(g7) & np.isnan(c7))
            result["bitwise_vs_cpu_oracle"] = {
                "rays": int(len(pick)), "rows": int(cnt - 1), "horizon_days": (cnt - 1) / 12.0,
                "identical_values_frac": float(same.mean()),
                "rays_identical_all_rows": int(same.all(axis=(0, 1)).sum()),
                "note": "GPU rows vs the oracle (NumPy, the reference's arithmetic) on the cpu_baseline sample"}
        if weak and world > 1:
            # not a BASELINE config (N x the C3 set): the aggregate rides under
            # its own key; the line's value stays empty
            result["weak_scaling"] = {"value": value, "unit": "ray-steps/s",
                                      "note": f"{world} x the C3 set (each rank its own seed grid); "
                                              "a diagnostic of per-GPU throughput, not BASELINE configs[3]"}
            result["value"] = None
        print(json.dumps(result))
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def backend_of(dist):
    return dist.get_backend() if dist is not None and dist.is_initialized() else None


def c5_parity_sample(eng, rows_all, fields, dev):
    """The C5 line's parity check: the 4 096-ray sample of
    tests/golden/c5_ref10_<storage>.npz (the oracle's TimeVaryingBackground,
    tools/make_c5_ref.py) integrated 10 days (41 levels) on this engine; every
    row must hash like the oracle's.  fp32 arithmetic (fp32a) is not the
    reference's: its positions are compared with the fp64 fixture instead."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_devmath import row_hashes
    g = np.load(os.path.join(ROOT, "tests", "golden", f"c5_ref10_{'fp64' if fields != 'fp32' else 'fp32'}.npz"))
    nt = int(g["nt"])
    idx = torch.as_tensor(g["idx"], device=dev)
    if rows_all.shape[1] != int(g["nslot"]):
        return {"skipped": "the sample indexes the 5-period C5 set"}
    r0 = rows_all[:, idx]
    got = {}
    eng.integrate(r0[:5].contiguous(), nt, 7200.0, ttotal=(nt - 1) * 7200.0, chunk=48,
                  sink=lambda a, b, o: got.__setitem__(a, o[:, :, :7].cpu().numpy().copy()))
    hist = np.full((7, nt, idx.numel()), np.nan)
    hist[:, 0] = r0.cpu().numpy()
    for a in sorted(got):
        hist[:, a:a + got[a].shape[1]] = np.transpose(got[a], (2, 1, 0))
    out = {"rays": int(idx.numel()), "rows": nt, "levels": int(g["nlev"]),
           "fixture": f"tests/golden/c5_ref10_{'fp64' if fields != 'fp32' else 'fp32'}.npz"}
    if fields == "fp32a":
        last = g["last"]
        ok = ~np.isnan(last[0]) & ~np.isnan(hist[0, -1])
        d = np.max(np.abs(hist[:2, -1, ok] - last[:2, ok]), axis=0) if ok.any() else np.zeros(1)
        out.update(vs="fp64-arithmetic oracle (fp32 RHS is not the reference's arithmetic)",
                   p50=float(np.median(d)), p99=float(np.percentile(d, 99)), max=float(d.max()),
                   alive_mismatch=int(np.sum(np.isnan(last[0]) != np.isnan(hist[0, -1]))))
    else:
        bad = int(np.sum(row_hashes(hist) != g["row_sha"]))
        out.update(rows_identical=nt - bad, bitwise=bad == 0)
    return out


def c5_rows_per_launch(fp32, world, nt):
    """C5's rows per launch of the long launches (before the memory cap).
    One GPU (round 5 final build, lane pairs and row-end reuse; one box):
    fp64 levels 96 rows (48 / 72 / 96 / 120 / 144: 1.54 / 1.59 / 1.61 / 1.59 /
    1.47e9 ray-steps/s -- each launch re-sorts the queue by cost class and
    grid cell, and the fp64 lookups gain from that locality), fp32 levels 360
    (240 / 360 / 540 / 1080: 1.56 / 1.59 / 1.46 / 1.49e9;
    profiles/r5/final4/c5_chunk_sweep.txt).  A split set runs the whole rest
    of the horizon in one launch (fp64, N = 2 / 4 / 8: 1.67-1.72 / 0.99 /
    0.78 s against 1.90 / 1.52 / 1.34 s at 96-row or 48-row launches: a
    shard's heaviest rays then run their chains without a barrier,
    profiles/r5/sched/c5_half_*.json; fp32 levels 8 shards 0.85 s against
    1.55 s at 240-row launches, profiles/r5/final4/c5_fp32_rehearsal*.json)
    -- except fp64 levels split 2 ways, whose shards are still throughput-bound:
    96 rows, 1.47 s against 1.54 s at 144 and 1.66 s in one launch (4 / 8
    shards at 96 rows: 1.27 / 1.09 s against 0.96 / 0.71 in one launch;
    profiles/r5/final5/c5_split_chunks.txt)."""
    if world > 1:
        return 96 if (world == 2 and not fp32) else nt - 1
    return 360 if fp32 else 96


def main_c5(args, dist, group, rank, world, dev, share=1):
    """BASELINE configs[4]: a 0.25-degree time-varying background (one level
    every 6 h, built on the device by rwrt_bs_ready, fp64 or fp32 storage) and
    1-degree global seeds x k = 1..10 x ``--c5-periods`` of the C3 periods,
    90 days at 2 h.  One step = GPU initial rows + the time-varying ray loop
    over the whole set (weak scaling: every rank its own C5 set, the seed grid
    shifted by rank x 1/N degree of longitude; strong: one set split like
    C3/C4, run_sharded); levels and sources are resident in HBM before the
    timed region (each rank builds the same levels from the same synthetic
    snapshots)."""
    from engine import RayEngine
    from levels import Levels
    from shard import broadcast_levels, run_sharded
    res, dt_bg = 0.25, 6 * 3600.0
    nt = int(round(args.days * 12)) + 1
    nlev = int(np.ceil((nt - 1) * 7200.0 / dt_bg)) + 1
    b0 = S.background_level(0, res=res)     # (the axes; every rank knows the grid)
    t_build = time.perf_counter()
    lv = Levels(b0["lat"], b0["lon"], nlev, t0=0.0, dt=dt_bg, fp32=(args.fields in ("fp32", "fp32a")), device=dev,
                arith32=(args.fields == "fp32a"))

    def make_uv(j):   # rank 0 only: the snapshots a real run reads from its file there
        bj = b0 if j == 0 else S.background_level(j, res=res)
        return bj["u"], bj["v"]
    # rank 0's u, v snapshots broadcast (RCCL over xGMI; gloo when ranks share a
    # GPU), every rank building its packed levels: outside the timed step
    bcast = broadcast_levels(lv, make_uv, group=group if dist else None)
    t_build = time.perf_counter() - t_build
    eng = RayEngine.from_levels(lv)
    cfg = S.config("C5")
    deg2rad = np.pi / 180.0
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    weak = args.scaling == "weak"
    offset = rank * cfg.dlon / world if weak else 0.0
    lon = (((cfg.SW_lon + offset) % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * deg2rad
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * deg2rad
    src = eng.sources(lon, lat)
    periods = S.C3_PERIODS_DAYS[: args.c5_periods]
    zcs = [eng.zwn_tensor(cfg.zwn, S.c3_freq(P)) for P in periods]
    rows = [None] * len(zcs)

    def make_y0():
        ys = []
        for j, zc in enumerate(zcs):
            rows[j], _ = eng.initial_rows_dev(src, zc, rows[j])
            ys.append(rows[j][:5].reshape(5, -1))
        return torch.cat(ys, dim=1)

    y0 = make_y0()
    nslot = y0.shape[1]
    n_live = int((~torch.isnan(y0.sum(0))).sum().item())
    # rows per launch: c5_rows_per_launch, capped by the row buffer's memory
    # (row blocks for the live rays only, as for C3)
    n_blk = n_live if weak else -(-n_live // world) + 2
    free = torch.cuda.mem_get_info(dev)[0] // share
    cap = max(1, min(nt - 1, int(0.8 * free) // (max(n_blk, 1) * 64)))
    chunk = min(args.chunk or c5_rows_per_launch(lv.fp32, 1 if weak else world, nt), cap)
    out = torch.empty((max(n_blk, 1), min(chunk, nt - 1), 8), dtype=torch.float64, device=dev)
    lead = [int(x) for x in str(args.first_chunk).split(",") if x]
    # latency mode (the time-varying latency waves: one ray per wave on its 64
    # lanes, BlockVaryingBG) for a split set's heaviest rays; one GPU's set is
    # throughput-bound
    team = 0 if (weak or world == 1) else (args.team if args.team == "auto" else
                                          (int(args.team.split(":")[0]), 1) if ":" in args.team else int(args.team))

    def one_step(events=None):
        if weak:
            return run_sharded(eng, make_y0(), nt, 7200.0, rank=0, world=1, probe=args.probe, lead=lead,
                               chunk=chunk, out=out, events=events, ttotal=(nt - 1) * 7200.0,
                               order_policy=args.order)
        return run_sharded(eng, make_y0(), nt, 7200.0, group=group, probe=args.probe, lead=lead,
                           chunk=chunk, out=out, events=events, ttotal=(nt - 1) * 7200.0,
                           order_policy=args.order, team=team, shard_probe=bool(args.shard_probe))

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    events, steps_done = [], 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = one_step(events)
        steps_done += r.steps_local
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rows_bytes = int(eng.rows_bytes)   # (the timed steps' row buffers; later sample runs reuse the engine)
    kern_s = sum(a.elapsed_time(b) for a, b in events) / 1e3
    rej = int(r.res.nrej.sum().item())
    tot_steps, max_el, tot_rej = steps_done, elapsed, rej
    if dist:
        t = torch.tensor([float(steps_done), elapsed, float(rej)], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        s, m = t.clone(), t.clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot_steps, max_el, tot_rej = s[0].item(), m[1].item(), s[2].item()
    if rank == 0:
        fbytes = 4 if lv.fp32 else 8
        bps = 6 * 4 * 11 * fbytes * 2          # 6 RHS x 4 corners x 11 fields x 2 levels
        per_launch_steps = steps_done / max(len(events), 1)
        avg_launch_s = kern_s / max(len(events), 1)
        workload = (f"C5: 1deg global seeds x k=1..10 x {len(periods)} periods, {args.days:g} d at 2 h, "
                    f"0.25deg time-varying background ({nlev} levels every 6 h, {args.fields} storage; "
                    f"BASELINE configs[4])")
        schedule = [args.probe] + [b - a for a, b in r.res.bounds]
        del out
        torch.cuda.empty_cache()
        parity = c5_parity_sample(eng, torch.cat([x.reshape(7, -1) for x in rows], dim=1), args.fields, dev) \
            if args.days >= 10 else {"skipped": "needs --days >= 10 (the fixture's horizon)"}
        c5_line = {
            "metric": METRIC, "value": tot_steps / max_el, "unit": "ray-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * max_el / args.steps,
            "higher_is_better": True, "scaling": "weak" if weak else "strong", "vs_baseline": None,
            "dtype": "f32 RHS, f64 stepper" if args.fields == "fp32a" else "f64",
            "data": "synthetic",
            "config": {"workload": workload, "ray_slots": nslot, "live_rays": n_live,
                       "rows": nt, "levels": nlev, "field_storage": args.fields,
                       "level_bytes": int(lv.packed[0].numel() * lv.packed.element_size()),
                       "rows_per_launch": chunk, "launch_rows": schedule,
                       "parallelism": (f"{world} rank(s), each its own C5 seed grid (shifted by rank/N deg)"
                                       if weak else f"one ray set over {world} GPU(s) (run_sharded, as C3/C4)")},
            "parity_sample_vs_oracle": parity,
            # the whole set's last rows (one set at every N when strong: the same hash at N = 1, 2, ..)
            "endpoints_rank0_sha256": endpoint_sha(r.endpoints) if (r.endpoints is not None and not weak) else None,
            "latency_mode": (f"{team if team == 'auto' else team} (time-varying latency waves: one ray per wave "
                             f"on its 64 lanes, BlockVaryingBG)" if team else "none"),
            "launches": [dict(d) for d in eng.launch_log],
            "rows_bytes": {"rank0": rows_bytes,
                           "note": "rank 0's device row buffer (row blocks for live rays only, ABI 4)"},
            "ray_steps_per_step": tot_steps / args.steps,
            "rejected_per_accepted": tot_rej * args.steps / max(tot_steps, 1),
            "levels_build_s": t_build,
            "levels_broadcast": dict(bcast, backend=backend_of(dist),
                                     note="rank 0's u, v snapshots (float32) broadcast in blocks of 16 levels, "
                                          "each rank building its packed levels with rwrt_bs_ready; before "
                                          "the timed steps (bs.py:202-262 reads the file on one process)"),
            "queue_order": args.order,
            "library_sha256": library_sha(),
            "init": "GPU rwrt_ray_initial inside every timed step",
            "roofline": roofline(per_launch_steps, avg_launch_s, workload, schedule, bps, args, bound="hbm",
                                 steps_per_s_gpu=tot_steps / max_el / world)}
        if weak and world > 1:
            c5_line["weak_scaling"] = {"value": c5_line["value"], "unit": "ray-steps/s",
                                       "note": f"{world} x the C5 set: a diagnostic, not BASELINE configs[4]"}
            c5_line["value"] = None
        print(json.dumps(c5_line))
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
