"""Where a live Lightning plot costs the LR driver's training thread.

python tools/diag/plot_stall.py [--batches 40] [--switch-us 0,500]

Runs ``apps/linear_regression.py`` on the GPU engine (1M-tweet wide batches)
with plotting off (unreachable Lightning), then on against a fake Lightning
in a child process, once per GIL switch interval given, and prints the
percentiles of the per-batch metrics: ``step_ms`` (train + report on the
training thread), ``call_ms`` (the engine call) and ``gil_wait_ms`` (the part
of the call after the engine returned, spent taking the GIL back).
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--switch-us", default="0")
    a = ap.parse_args()
    from fakes import FakeLightningProcess
    from twitter_stream_ml_amd.apps import linear_regression as app
    base = ["--master", "rocm[1]", "--twtweb", "http://127.0.0.1:9", "--source", "replay:synthetic:wide:4",
            "--seconds", "0", "--batchSize", "1000000", "--sourceRate", "0", "--numBatches", str(a.batches),
            "-f", "1000000"]
    default_si = sys.getswitchinterval()

    def run(tag, lightning, si_us):
        sys.setswitchinterval(si_us / 1e6 if si_us > 0 else default_si)
        path = os.path.join(tempfile.mkdtemp(), "m.jsonl")
        os.environ["TWTML_METRICS"] = path
        assert app.main(base + ["--lightning", lightning]) == 0
        recs = [json.loads(l) for l in open(path)]
        recs = [r for r in recs if "step_ms" in r][8:]
        out = {"run": tag, "switch_us": si_us or default_si * 1e6}
        for k in ("step_ms", "call_ms", "gil_wait_ms", "train_ms"):
            v = np.array([r.get(k, np.nan) for r in recs], float)
            out[k] = {"p50": round(float(np.nanpercentile(v, 50)), 3), "p90": round(float(np.nanpercentile(v, 90)), 3),
                      "p99": round(float(np.nanpercentile(v, 99)), 3), "max": round(float(np.nanmax(v)), 3)}
        print(json.dumps(out), flush=True)

    sis = [int(x) for x in a.switch_us.split(",")]
    run("off", "http://127.0.0.1:9", sis[0])
    lgn = FakeLightningProcess().start()
    try:
        for si in sis:
            run("on", lgn.url, si)
        print(json.dumps({"lightning": lgn.summary()}), flush=True)
    finally:
        lgn.stop()


if __name__ == "__main__":
    main()
