"""bench.py --master local[N]: BASELINE.json config 1 (the reference's own
CPU mode, ConfArguments.scala:54-56) -- the line vs_baseline is measured
against (profiles/r6/config1_local2.json).  CPU only."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_local_bench_line():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--master", "local[2]", "--steps", "2",
                        "--warmup", "1", "--batch", "3000", "--profile", "bench", "--features", "1000"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "p50_microbatch_latency_ms"):
        assert k in d, k
    assert d["n_gpus"] == 0 and d["dtype"] == "fp64" and d["steps"] == 2
    assert d["config"]["parallelism"] == "cpu local[2]" and d["config"]["global_batch"] == 3000
    assert d["value"] > 0 and d["p50_microbatch_latency_ms"] > 0 and d["host_threads"] == 1
    assert d["trained_tweets_per_step"] > 0


def test_cpu_local_bench_rejects_other_masters():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--master", "yarn"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "local[N]" in p.stderr
