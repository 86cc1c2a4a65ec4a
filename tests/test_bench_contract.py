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
