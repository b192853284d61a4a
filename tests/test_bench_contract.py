"""bench.py driver contract on CPU: exactly one JSON line from rank 0 with the BASELINE.json metric,
for a single process and for a 2-rank torch.distributed.run (gloo) launch — the same launch line the
driver uses on an 8-GPU node; ``--gpus N`` without a launcher must start N ranks (never measure one in
their place); a hung rank must end the whole job non-zero in bounded time (progress watchdog)."""
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, env_extra=None):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out), sorted(KEYS - set(out))
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert out["metric"] == json.load(f)["metric"]
    assert out["value"] > 0 and out["higher_is_better"] is True
    assert out["steps"] == 20 and out["warmup"] == 2
    return out


def test_bench_single_process():
    out = _run([sys.executable, "bench.py", "--steps", "20", "--warmup", "2"])
    assert out["config"]["parallelism"].endswith("p1 (1x1)")
    # the init-time prediction next to the measurement (HIP engines measure one; the CPU backend does not)
    assert "sched_predicted_us_per_gen" in out and "predicted_over_measured" in out
    if out["config"]["backend"] == "hip":
        assert out["sched_predicted_us_per_gen"] > 0 and out["predicted_over_measured"] > 0, out
    else:
        assert out["sched_predicted_us_per_gen"] is None and out["predicted_over_measured"] is None


def test_bench_prediction_fields():
    sys.path.insert(0, REPO)
    import bench

    f = bench.prediction_fields(11.0, 11.2)
    assert f == {"sched_predicted_us_per_gen": 11.0, "predicted_over_measured": round(11.0 / 11.2, 4)}
    assert bench.prediction_fields(0.0, 11.2) == {"sched_predicted_us_per_gen": None, "predicted_over_measured": None}
    assert bench.prediction_fields(None, 11.2)["sched_predicted_us_per_gen"] is None


def test_bench_torchrun_two_ranks():
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                "--steps", "20", "--warmup", "2"])
    cfg = out["config"]
    assert cfg["parallelism"].endswith("p2 (1x2)")
    # per-rank diagnosis arrays, one entry per rank, consistent with the aggregates
    pr = out["per_rank"]
    for key in ("per_rank_elapsed_us", "per_rank_t0_offset_us", "per_rank_exchange_us", "per_rank_superstep_us",
                "per_rank_schedule", "per_rank_kernel", "per_rank_depth"):
        assert len(pr[key]) == 2, (key, pr)
    assert max(pr["per_rank_elapsed_us"]) == out["timing"]["per_rank_elapsed_max_us"]
    assert min(pr["per_rank_t0_offset_us"]) == 0 and len(set(pr["per_rank_schedule"])) == 1
    # weak scaling: every rank owns a full tile, the global board grows with the rank count
    assert cfg["board"][0] == 2 * cfg["tile_per_rank"][0]


def test_bench_reports_start_skew():
    out = _run([sys.executable, "bench.py", "--steps", "20", "--warmup", "2"])
    assert out["start_skew_us"] >= 0
    assert out["timing"]["per_rank_elapsed_max_us"] > 0


def test_bench_without_launcher_starts_the_ranks():
    """The driver's --gpus N run, mis-launched as a plain process, still measures N ranks."""
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "2"])
    assert out["config"]["parallelism"].endswith("p2 (1x2)")
    assert out["config"]["board"][0] == 2 * out["config"]["tile_per_rank"][0]


def test_bench_rank_count_mismatch_fails():
    env = dict(os.environ, OMP_NUM_THREADS="1", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "4", "--warmup", "1"], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # the one-JSON-line contract holds for the failure too
    rec = json.loads(lines[0])
    assert rec["value"] is None and "WORLD_SIZE=1" in rec["error"] and rec["n_gpus"] == 1


def test_bench_hung_rank_ends_the_job():
    """GOL_FAULT hangs rank 1 inside its run: its watchdog aborts it (exit 4) and the launcher ends the
    job non-zero within a bounded time, instead of the job hanging until the driver's timeout."""
    env = dict(os.environ, OMP_NUM_THREADS="1", GOL_FAULT="1:10:hang")
    env.pop("WORLD_SIZE", None)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                        "--steps", "20", "--warmup", "2", "--watchdog", "3"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    dt = time.monotonic() - t0
    assert r.returncode != 0
    assert "watchdog" in r.stderr
    assert dt < 120, dt


def test_bench_rank_problems():
    """The checks that turn a multi-rank record into an error record (non-zero exit, value null)."""
    sys.path.insert(0, REPO)
    import bench

    same = [{"schedule": "full+subtiles2ov", "kernel": "temporal", "depth": 128}] * 4
    assert bench.rank_problems(same, 4, 4) == []
    assert bench.rank_problems(same, 4, None) == []  # host transport: no communicator to check
    diff = same[:3] + [{"schedule": "full+subtiles2", "kernel": "temporal", "depth": 128}]
    (p,) = bench.rank_problems(diff, 4, 4)
    assert "disagree" in p and "3:full+subtiles2/temporal/128" in p
    # a per-rank kernel choice is reported, not an error; a halo depth mismatch is
    kern = same[:3] + [{"schedule": "full+subtiles2ov", "kernel": "pipe@24", "depth": 128}]
    assert bench.rank_problems(kern, 4, 4) == []
    (p,) = bench.rank_problems(same[:3] + [{"schedule": "full+subtiles2ov", "kernel": "temporal", "depth": 64}], 4, 4)
    assert "disagree" in p
    (p,) = bench.rank_problems(same, 4, 2)
    assert "spans 2 of 4" in p


def test_bench_stdout_is_the_record_only():
    """Writes to file descriptor 1 from C libraries (RCCL's version block at communicator init) must not
    reach stdout: bench.py points fd 1 at stderr and keeps its own handle for the JSON line."""
    code = (
        "import os, sys; sys.path.insert(0, %r); import bench; "
        "bench._RECORD = bench._reserve_stdout(); "
        "os.write(1, b'RCCL version : banner\\n'); print('python print'); "
        "bench.emit({'metric': 'm', 'value': 1})" % REPO
    )
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert lines == ['{"metric": "m", "value": 1}'], r.stdout
    assert "RCCL version" in r.stderr and "python print" in r.stderr
