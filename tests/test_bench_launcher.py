"""bench.py's N-GPU launcher (CPU): ``--gpus N`` without a launcher starts N
ranks itself; under torch.distributed.run it checks N against WORLD_SIZE.

The driver runs ``python bench.py --gpus N`` (or the same under
torch.distributed.run); either must give an N-rank run whose rank 0 prints
one line with ``n_gpus: N`` (``--gpus`` used to be ignored).
``--dry-run`` stops after the process group is up, so the spawn path is
tested end to end here with gloo (no GPU).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_resolve_world_rules():
    from bench import resolve_world
    assert resolve_world(None, {}) == ("rank", 1)
    assert resolve_world(1, {}) == ("rank", 1)
    assert resolve_world(8, {}) == ("spawn", 8)
    assert resolve_world(4, {"WORLD_SIZE": "4"}) == ("rank", 4)
    assert resolve_world(None, {"WORLD_SIZE": "2"}) == ("rank", 2)
    with pytest.raises(SystemExit):
        resolve_world(8, {"WORLD_SIZE": "2"})          # --gpus disagrees with the launcher
    with pytest.raises(SystemExit):
        resolve_world(0, {})


def _bench(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", **(env_extra or {}))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


def test_gpus2_spawns_two_ranks_one_line():
    p, lines = _bench(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout                # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_sum"] == 2.0 and d["backend"] == "gloo"
    # the default N > 1 run is BASELINE configs[3]: ONE C3 set split over the
    # ranks (strong scaling); weak scaling is an explicit, separately keyed
    # diagnostic
    assert d["scaling"] == "strong"


def test_weak_scaling_is_opt_in():
    p, lines = _bench(["--gpus", "2", "--dry-run", "--scaling", "weak"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(lines[0])["scaling"] == "weak"


def test_gpus_mismatch_under_launcher_fails_loudly():
    p, lines = _bench(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and not lines
    assert "WORLD_SIZE=2" in p.stderr


def test_failing_rank_ends_the_run():
    # an unreachable rendezvous makes every rank fail: the parent must return
    # non-zero instead of hanging
    p, lines = _bench(["--gpus", "2", "--dry-run"], {"RWRT_DIST_BACKEND": "no_such_backend"})
    assert p.returncode != 0 and not lines


def test_roofline_hbm_bound_for_c5(tmp_path):
    """C5 lines lead with the HBM roofline (PMC line traffic per launch over
    the launch time) and keep the VALU-issue figures beside it."""
    import json
    import bench
    prof = {"workload": "w", "launch_rows": [6, 24], "library_sha256": "x", "valu_insts_per_launch": 1e9,
            "clock_hz": 2.4e9, "simds": 1024, "cycles_per_valu": 4}
    traf = dict(prof, traffic_bytes_per_launch=4e11)
    (tmp_path / "valu.json").write_text(json.dumps(prof))
    (tmp_path / "traffic.json").write_text(json.dumps(traf))

    class A:
        valu_profile = str(tmp_path / "valu.json")
        traffic = str(tmp_path / "traffic.json")
    r = bench.roofline(1e6, 0.1, "w", [6, 24], 4224, A, bound="hbm")
    assert r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert abs(r["achieved"] - 4000.0) < 1e-6 and abs(r["frac"] - 0.5) < 1e-9
    assert abs(r["valu_issue"]["frac"] - 1e9 / 0.1 / (1024 * 2.4e9 / 4)) < 1e-9
    v = bench.roofline(1e6, 0.1, "w", [6, 24], 2112, A)
    assert v["bound"] == "valu_issue" and v["hbm"]["frac"] == r["frac"]


def test_schedule_defaults():
    """The bench's schedule defaults by what one GPU holds (a whole C3 set,
    zonal or not, a split one, C5); explicit values are kept."""
    import argparse
    import bench

    def ns(**kw):
        base = dict(config="C3", scaling="weak", bg="zonal", first_chunk=None, probe=None, team=None)
        base.update(kw)
        return argparse.Namespace(**base)
    a = bench.schedule_defaults(ns(), 1)
    assert (a.first_chunk, a.probe, a.team) == ("24,160", 4, "64,64,64")
    a = bench.schedule_defaults(ns(bg="nonzonal"), 8)
    assert (a.first_chunk, a.probe, a.team) == ("24,160", 4, "0")
    a = bench.schedule_defaults(ns(scaling="strong"), 8)
    assert (a.first_chunk, a.probe, a.team) == ("96", 6, "auto")
    a = bench.schedule_defaults(ns(scaling="strong"), 1)
    assert (a.first_chunk, a.probe, a.team) == ("24,160", 4, "64,64,64")
    # C5: no latency mode by default (its launch-ending rays are not predictable)
    a = bench.schedule_defaults(ns(config="C5"), 1)
    assert (a.first_chunk, a.probe, a.team) == ("24,96", 6, "0")
    a = bench.schedule_defaults(ns(probe=6, team="0", first_chunk="24"), 1)
    assert (a.first_chunk, a.probe, a.team) == ("24", 6, "0")


def test_split_argument():
    """--split: 'off', 'auto' (one cut after RayEngine.SPLIT_ROWS) or 'auto:a,b,..'
    (cuts after a, a+b, .. rows; profiles/r4/sched/nonzonal_split.txt)."""
    import argparse
    from bench import _split_arg
    for ok in ("off", "auto", "auto:300", "auto:300,300"):
        assert _split_arg(ok) == ok
    for bad in ("on", "auto:", "auto:0", "auto:300,x", "auto:-5", "off:3", "auto:~prev"):
        with pytest.raises(argparse.ArgumentTypeError):
            _split_arg(bad)
