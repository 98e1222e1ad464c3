#!/bin/bash
# Every bench line of the README "Performance" table on one box, one after the
# other (JSON -> gpurun_out/final/<name>.json), then the real driver replay.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=final STEP_TIMEOUT=400 bash tools/gpu_run.sh \
  "bench:wide@--steps 20 --warmup 5" \
  "bench:toy@--profile bench --steps 20 --warmup 5" \
  "bench:kmeans@--model kmeans --steps 20 --warmup 5" \
  "bench:kmeans_k3@--model kmeans --k 3 --text-dims 0 --steps 20 --warmup 5" \
  "bench:kmeans_prepacked@--model kmeans --prepacked --steps 20 --warmup 5" \
  "bench:wide100m@--features 100000000 --hash murmur3 --steps 20 --warmup 5" \
  "bench:prepacked@--prepacked --steps 20 --warmup 5" \
  "bench:forced_dp@--force-dp --steps 20 --warmup 5" || exit $?
bash tools/app_replay.sh
