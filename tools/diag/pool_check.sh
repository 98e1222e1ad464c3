# Staging changes: GPU tests that stage batches, the staging breakdown, and
# the host-bound (k-means k=3 d=2) and PCIe-bound (LR toy) bench lines.
bash tools/gpu_tests.sh -k "lr_engine or kmeans or apps or bench or sizing" && \
PYTHONPATH=. timeout -k 10 300 python tools/diag/stage_time.py && \
timeout -k 10 300 python bench.py --model kmeans --k 3 --text-dims 0 --steps 20 --warmup 5 > gpurun_out/b_km3.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/b_def.log 2>&1 && \
grep -h metric gpurun_out/b_km3.log gpurun_out/b_def.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config']['model'][:40], round(d['value']/1e6,1), d['ms_per_step'], d.get('host_stage_ms_p50'), d.get('device_ms_mean'))"
