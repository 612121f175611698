"""bench.py's host logic on the CPU: the N-rank self-launch, the world-size check, and the PMC
staleness rule (no GPU work: --probe-dist stops after the process group is up)."""
import importlib.util
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _bench_module():
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(RT_BENCH_BACKEND="gloo", **kw)
    return env


def test_gpus_2_without_a_launcher_runs_two_ranks():
    """`python bench.py --gpus 2` (as the driver runs it) starts 2 ranks itself: n_gpus 2, world 2."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--probe-dist"], capture_output=True, text=True,
                       env=_env(), timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["dist"]["world_size_initialised"] == 2
    assert line["dist"]["ranks"] == [0, 1]


def test_world_size_mismatch_exits_nonzero():
    """A rank whose world is not --gpus refuses to report (no silent 1-GPU line labelled N GPUs)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--probe-dist"], capture_output=True, text=True,
                       env=_env(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                MASTER_PORT="29517"), timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_pmc_record_from_other_sources_is_stale():
    b = _bench_module()
    rec = {"hbm_bytes_per_launch": 4.7e10, "valu_busy": 0.63, "commit": "656c11f74452", "src_hash": "aaaaaaaaaaaa",
           "launch_ms": 39.5, "issue_frac": 0.91, "issue_frac_vs_ubench": 1.01, "pmc_flop_frac": 0.27}
    f = b.pmc_fields(rec, "bbbbbbbbbbbb", "profiles/pmc.json")
    assert f["pmc_source"]["stale"] is True and f["traffic"] is None and f["valu_busy"] is None
    assert f["issue_frac"] is None and f["pmc_flop_frac"] is None
    f = b.pmc_fields(rec, "aaaaaaaaaaaa", "profiles/pmc.json")
    assert f["pmc_source"]["stale"] is False and f["traffic"] == 4.7e10 and f["valu_busy"] == 0.63
    assert f["issue_frac"] == 0.91 and f["issue_frac_vs_ubench"] == 1.01 and f["pmc_flop_frac"] == 0.27
    old = dict(rec)
    del old["src_hash"]   # a record written before the hash existed
    assert b.pmc_fields(old, "aaaaaaaaaaaa", "x")["pmc_source"]["stale"] is True
    assert b.pmc_fields({}, "aaaaaaaaaaaa", "x") == {"traffic": None, "valu_busy": None, "issue_frac": None,
                                                     "issue_frac_vs_ubench": None, "pmc_flop_frac": None,
                                                     "pmc_source": None}
