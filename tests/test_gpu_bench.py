"""bench.py contract on one MI355X: one JSON line with the driver's fields,
the end-to-end default, the pre-packed device pipeline and the config-5 HBM
micro-batch sizing (``--batch hbm``, ops/sizing.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
          "scaling", "vs_baseline", "dtype", "data", "config"}


def _bench(*args):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert FIELDS <= set(d), FIELDS - set(d)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["higher_is_better"] is True
    return d


@pytest.mark.parametrize("mode", [[], ["--prepacked"]], ids=["e2e", "prepacked"])
def test_bench_json_line(hip_module, mode):
    d = _bench("--batch", "100000", "--steps", "3", "--warmup", "1", "--pool", "2", *mode)
    assert d["steps"] == 3 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 100000
    assert ("e2e" in d["ingest"]) == (not mode)
    # the timed window starts with an empty pipeline
    assert d["prestaged_at_t0"] == 0
    assert d["comm_world"] == 1 and len(d["per_rank_value"]) == 1
    assert d["per_rank_host"][0]["pinned_mb"] > 0
    # the window's H2D bytes (engine counter, ~150-200 B per wide tweet) and
    # the host-link floor they imply at this box's measured pinned bandwidth
    assert 100 < d["h2d_bytes_per_tweet"] < 400, d["h2d_bytes_per_tweet"]
    assert 20 < d["h2d_gbps"] < 200 and 0 < d["h2d_floor_ms_per_step"] <= d["ms_per_step"] * 1.05


def test_bench_force_dp_reports_the_collective(hip_module):
    """--force-dp: the engine's DP path through a world-1 RCCL communicator;
    the JSON shows the gradient all-reduces per step and their time."""
    d = _bench("--batch", "100000", "--steps", "3", "--warmup", "1", "--pool", "2", "--force-dp")
    assert d["config"]["parallelism"] == "dp1-forced" and d["comm_kind"] == "rccl"
    assert d["comm_world"] == 1 and d["grad_allreduce_per_step"] >= 1
    assert d["grad_allreduce_us_per_iter"] > 0
    assert d["comm_counters"]["allgather_calls"] >= 3 + 1


def test_bench_hbm_batch_sizing(hip_module):
    d = _bench("--batch", "hbm", "--batch-cap", "131072", "--steps", "2", "--warmup", "1", "--pool", "2")
    s = d["config"]["batch_sizing"]
    assert s["hbm_max_rows"] >= 131072          # 288 GB holds far more than the cap
    assert d["config"]["global_batch"] == 131072
