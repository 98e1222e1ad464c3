"""Shared pytest configuration.

Markers: ``gpu`` -- needs a real MI355X (the driver runs ``-m gpu`` on a GPU
box and ``-m "not gpu"`` here).  The test "classpath" for application.conf is
tests/resources (like sbt's src/test/resources).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
os.environ.setdefault("TWTML_CONFIG_PATH", os.path.join(ROOT, "tests", "resources"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def hip_module():
    """The HIP engine extension; GPU tests fail loudly if it cannot load."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU visible")
    from twitter_stream_ml_amd.ops import _native
    return _native.hip()


@pytest.fixture(autouse=True)
def _engine_teardown_clean(request):
    """GPU tests: a device error that an engine destructor found (its last
    work faulted; csrc/hip/debug.h) fails the test that owned the engine,
    not whichever test touches the device next."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc
    gc.collect()
    from twitter_stream_ml_amd.ops import _native
    try:
        errs = list(_native.hip().teardown_errors())
    except Exception:   # noqa: BLE001 -- the extension is not loaded: nothing to check
        return
    assert not errs, f"engine teardown found device errors: {errs}"


# Timing gates of the GPU suite (p99 bounds on a shared box) record their
# measured value and bound here; the terminal summary prints them for every
# run, passing or not, so the suite output carries each gate's headroom.
_MARGINS = []


@pytest.fixture
def timing_margin():
    def record(name, measured, bound, unit="ms"):
        _MARGINS.append((name, float(measured), float(bound), unit))
    return record


def pytest_terminal_summary(terminalreporter):
    if not _MARGINS:
        return
    terminalreporter.section("timing gates (measured vs bound)")
    for name, m, b, unit in _MARGINS:
        head = 100.0 * (b - m) / b if b else float("nan")
        terminalreporter.write_line(f"{name}: {m:.3f} {unit} vs bound {b:.3f} {unit} ({head:+.1f} % headroom)")
