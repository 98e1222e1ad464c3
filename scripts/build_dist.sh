#!/bin/bash
# Distribution archive (the reference's build.sh): compiled in-tree extensions
# for gfx950 + package + configs + web assets, as twtml-mi355x-<version>.tar.gz.
set -euo pipefail
cd "$(dirname "$0")/.."
python -m twitter_stream_ml_amd._build
VER=$(python -c "import twitter_stream_ml_amd as t; print(t.__version__)")
OUT=dist/twtml-mi355x-$VER
rm -rf "$OUT" && mkdir -p "$OUT"
cp -r twitter_stream_ml_amd "$OUT/"
find "$OUT" -name __pycache__ -prune -exec rm -rf {} +
cp README.md pyproject.toml Procfile app.json bench.py "$OUT/"
tar -C dist -czf "dist/twtml-mi355x-$VER.tar.gz" "twtml-mi355x-$VER"
echo "dist/twtml-mi355x-$VER.tar.gz"
