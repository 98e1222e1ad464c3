"""Dashboard JavaScript run under node with a fake DOM (skipped without node).

``web/assets/js/embed.js`` speaks the pym.js 0.4.5 protocol the reference
dashboard vendors (``web/src/main/assets/lib/pym/pym.js:132-585``): iframe
URL parameters, parent ``width`` on load / resize, child ``height`` and
``navigateTo``, id and origin filtering (``tests/js/embed_test.js``).
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_embed_pym_protocol():
    p = subprocess.run(["node", os.path.join(HERE, "js", "embed_test.js")], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "embed.js ok" in p.stdout
