"""Prep-stream tuning knobs keep the model unchanged.

``TWTML_PREP_SLICES`` (prep kernels in chunk-range launches),
``TWTML_PREP_WG_MULT`` (grid caps of the grid-stride prep kernels) and
``TWTML_PREP_CU`` (CU-masked prep stream) only change how batch t+1's
preparation is launched (``profiles/README.md``, prep / GD-loop
interference).  The engine reads them once per process, so the knob run is a
subprocess; it trains the same tiered (wide) and hybrid (toy) batches as the
in-process default engine and the weights must agree.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NOW = 1_700_000_000_000
CASES = [("wide", 1 << 20, 20000, 2), ("twitter", 1 << 20, 6000, 2)]

SCRIPT = r"""
import json, sys
import numpy as np
import torch  # noqa: F401
sys.path.insert(0, {root!r})
from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
out = {{}}
for ci, (profile, F, rows, nb) in enumerate({cases!r}):
    eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=F, max_rows=rows, max_units=rows * 300,
                                                num_iterations=20), device=0)
    synth = SynthConfig.profile(profile, seed=70 + ci)
    batches = [generate_batch(synth, t * rows, rows, batch_time_ms={now} + t * 5000) for t in range(nb)]
    for b in batches[:eng.raw_slots - 1]:
        eng.prefetch(b)
    its = [eng.train_batch(b, want_pred=False)["iterations"] for b in batches]
    np.save(sys.argv[1] + f"/w{{ci}}.npy", eng.get_weights())
    out[ci] = its
print(json.dumps(out))
"""


def test_prep_knobs_leave_the_model_unchanged(tmp_path, hip_module):
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    env = dict(os.environ, TWTML_PREP_SLICES="3", TWTML_PREP_WG_MULT="2", TWTML_PREP_CU="7:8")
    code = SCRIPT.format(root=ROOT, cases=CASES, now=NOW)
    p = subprocess.run([sys.executable, "-c", code, str(tmp_path)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    its_knob = json.loads(p.stdout.strip().splitlines()[-1])
    for ci, (profile, F, rows, nb) in enumerate(CASES):
        eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=F, max_rows=rows, max_units=rows * 300,
                                                    num_iterations=20), device=0)
        synth = SynthConfig.profile(profile, seed=70 + ci)
        its = [eng.train_batch(generate_batch(synth, t * rows, rows, batch_time_ms=NOW + t * 5000),
                               want_pred=False)["iterations"] for t in range(nb)]
        assert its == its_knob[str(ci)], (profile, its, its_knob[str(ci)])
        w = eng.get_weights()
        wk = np.load(tmp_path / f"w{ci}.npy")
        # far-forward row sums use LDS float atomics (order may differ run to run)
        np.testing.assert_allclose(wk, w, rtol=1e-6, atol=1e-9 * max(np.abs(w).max(), 1e-12))
