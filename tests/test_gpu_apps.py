"""End-to-end drivers on the MI355X engine (``--master rocm[1]``).

The same CLI run on the CPU engine (``local[1]``) and on the GPU engine must
produce the same model: LR weights agree to fp32-engine tolerance, k-means
centres/weights closely (split-cluster ties aside, see test_gpu_kmeans).
"""
import numpy as np
import pytest

from twitter_stream_ml_amd.checkpoint import load_kmeans, load_linear_regression, load_progress

pytestmark = pytest.mark.gpu


def _lr_args(master, ck):
    return ["--master", master, "--lightning", "http://127.0.0.1:9", "--twtweb", "http://127.0.0.1:9",
            "--seconds", "0", "--batchSize", "3000", "--sourceRate", "0", "--numBatches", "4",
            "-f", "2048", "-i", "20", "--checkpoint", str(ck), "--checkpointInterval", "2"]


def test_lr_driver_gpu_matches_cpu(hip_module, tmp_path):
    from twitter_stream_ml_amd.apps import linear_regression as app
    assert app.main(_lr_args("local[1]", tmp_path / "cpu")) == 0
    assert app.main(_lr_args("rocm[1]", tmp_path / "gpu")) == 0
    w_cpu, _ = load_linear_regression(str(tmp_path / "cpu"))
    w_gpu, _ = load_linear_regression(str(tmp_path / "gpu"))
    assert load_progress(str(tmp_path / "gpu"))["batches"] == 4
    scale = np.abs(w_cpu[:-1]).max()
    np.testing.assert_allclose(w_gpu[:-1], w_cpu[:-1], rtol=2e-3, atol=2e-4 * scale)


def test_lr_driver_gpu_resume_auto(hip_module, tmp_path):
    from twitter_stream_ml_amd.apps import linear_regression as app
    ck = tmp_path / "ck"
    args = _lr_args("rocm[1]", ck)
    args[args.index("--numBatches") + 1] = "2"
    assert app.main(args) == 0
    assert load_progress(str(ck))["batches"] == 2
    args[args.index("--numBatches") + 1] = "4"
    assert app.main(args + ["--resume", "auto"]) == 0
    assert load_progress(str(ck))["batches"] == 4


def test_kmeans_driver_gpu_matches_cpu(hip_module, tmp_path):
    from twitter_stream_ml_amd.apps import kmeans as app
    base = ["--seconds", "0", "--batchSize", "2500", "--sourceRate", "0", "--numBatches", "3",
            "--k", "3", "--checkpointInterval", "1"]
    assert app.main(base + ["--master", "local[1]", "--checkpoint", str(tmp_path / "cpu")]) == 0
    assert app.main(base + ["--master", "rocm[1]", "--checkpoint", str(tmp_path / "gpu")]) == 0
    c_cpu, w_cpu = load_kmeans(str(tmp_path / "cpu"))
    c_gpu, w_gpu = load_kmeans(str(tmp_path / "gpu"))
    np.testing.assert_allclose(w_gpu.sum(), w_cpu.sum(), rtol=1e-9)
    assert np.abs(w_gpu - w_cpu).sum() <= 0.01 * w_cpu.sum()
    np.testing.assert_allclose(c_gpu, c_cpu, rtol=0.05, atol=0.05)
