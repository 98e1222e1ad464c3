"""Kernels per HIP stream from a rocprofv3 kernel trace CSV:
python tools/diag/stream_kernels.py run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(collections.Counter)
for r in rows:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    name = re.sub(r"\(.*$", "", name).replace("void ", "").replace("twtml::", "")
    by[(r["Agent_Id"], r["Queue_Id"], r["Stream_Id"])][name] += 1
PREP = re.compile(r"k_cesu|k_featurize|k_remap|k_tier|k_far_csc|k_code_table|k_hot_select|k_row_normalize|"
                  r"k_filter|k_sort|k_union|k_compact|k_pack_c1|k_batch_bounds")
for key, cnt in sorted(by.items(), key=lambda kv: -sum(kv[1].values())):
    prep = sum(v for k, v in cnt.items() if PREP.search(k))
    gd = sum(v for k, v in cnt.items() if re.search(r"k_sgd_|k_far_grad", k))
    print(f"agent {key[0]} queue {key[1]} stream {key[2]}: {sum(cnt.values())} dispatches, "
          f"GD-loop kernels {gd}, prep kernels {prep}")
    for k, v in cnt.most_common(14):
        print(f"    {v:6d}  {k}")
