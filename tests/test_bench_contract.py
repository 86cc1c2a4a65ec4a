"""bench.py's JSON line keeps the driver's contract (one line; metric/value/unit/n_gpus/steps/
warmup/ms_per_step/higher_is_better/scaling/vs_baseline/dtype/data/config) plus the roofline,
cpu_baseline and parity objects. Runs bench.py as a child process on the GPU at a tiny step count."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line_contract():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
                          "--cpu-budget", "2"], capture_output=True, text=True, timeout=110, cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k, t in (("metric", str), ("value", float), ("unit", str), ("n_gpus", int), ("steps", int), ("warmup", int),
                 ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str), ("dtype", str), ("data", str),
                 ("config", dict), ("roofline", dict), ("cpu_baseline", dict), ("parity", dict)):
        assert isinstance(d[k], t), k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["vs_baseline"] is None and "workload" in d["config"]
    r = d["roofline"]
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s" and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0 and c["sample"]
    ct = d["cpu_baseline_torch"]
    assert ct["autograd"] is True and ct["value"] > 0 and ct["cores"] >= 1
    assert d["parity"]["return_max_rel_err"] < 1e-5
    assert [v["precision"] for v in d["variants"]] == ["f16x6", "f16x3"]


def test_launch_ranks_starts_one_process_per_rank(tmp_path):
    """bench.py --gpus N without a launcher: N children with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    and the parent's argv; a failing rank's status comes back (CPU, a stub script stands in)."""
    sys.path.insert(0, REPO)
    import bench
    stub = tmp_path / "stub.py"
    stub.write_text("import os, sys\n"
                    "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')\n"
                    "open(os.path.join(sys.argv[1], 'r' + os.environ['RANK']), 'w').write("
                    "' '.join(os.environ[k] for k in keys) + ' ' + ' '.join(sys.argv[2:]))\n"
                    "sys.exit(3 if os.environ['RANK'] == sys.argv[2] else 0)\n")
    assert bench.launch_ranks(3, str(stub), [str(tmp_path), "-1", "--x"]) == 0
    got = sorted((tmp_path / f"r{r}").read_text().split() for r in range(3))
    assert [g[:3] for g in got] == [["0", "0", "3"], ["1", "1", "3"], ["2", "2", "3"]]
    assert {g[3] for g in got} == {"127.0.0.1"} and len({g[4] for g in got}) == 1
    assert all(g[5:] == ["-1", "--x"] for g in got)
    assert bench.launch_ranks(2, str(stub), [str(tmp_path), "1"]) == 3


@pytest.mark.gpu
def test_bench_gpus_2_launches_two_ranks():
    """`bench.py --gpus 2` launches its own two ranks (gloo here: one GPU on this box, both ranks share
    it); the line reports n_gpus 2, the process-group world size, and the strong walker split."""
    env = dict(os.environ, MBRL_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
                          "--warmup", "1", "--no-variants", "--no-cpu-baseline"], capture_output=True, text=True,
                         timeout=110, cwd=REPO, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["world_size"] == 2 and d["config"]["backend"] == "gloo"
    assert d["config"]["candidates_per_gpu"] == 4096 and d["scaling"] == "weak"
    assert d["strong"]["candidates_per_gpu"] == 8192 and d["strong"]["n_gpus"] == 2


@pytest.mark.gpu
def test_bench_gpus_8_launches_eight_ranks():
    """The driver's SCALE node runs `bench.py --gpus 8`: the 8-rank line is produced here first, eight
    rank processes over gloo sharing this box's one GPU (the N = 8 sharded protocol, the weak line at
    4096 candidates per rank, the walker split at 2048 and the headline split at 512 per rank)."""
    env = dict(os.environ, MBRL_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "2",
                          "--warmup", "1", "--no-variants", "--no-cpu-baseline"], capture_output=True, text=True,
                         timeout=280, cwd=REPO, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["world_size"] == 8 and d["config"]["backend"] == "gloo"
    assert d["config"]["candidates_per_gpu"] == 4096 and d["scaling"] == "weak"
    assert d["strong"]["candidates_per_gpu"] == 2048 and d["strong"]["n_gpus"] == 8
    assert d["strong_headline"]["candidates_per_gpu"] == 512 and d["strong_headline"]["n_gpus"] == 8
    assert d["plan_gpu_ms"] > 0 and d["value"] > 0 and d["roofline"]["frac"] > 0
