"""Summarize a rocprofv3 --kernel-trace --stats run of the default bench into the per-launch
duration bench.py reports beside its live HIP-event figure (profiles/<round>/rocprof_bench.json).

  python tools/rocprof_summary.py gpurun_out/prof_bench profiles/r04/rocprof_bench.json

One hot-path launch of the headline is the generated k_all_<model> plus the work-list
constraint kernel; their per-dispatch average durations (AverageNs of the stats table, which
counts each dispatch from its own start to its own end) are summed. The record is keyed by
codegen.source_hash, so bench.py only uses it for the kernel it was measured on.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(src, dst, model="humanoid"):
  from mujoco_inversedynamicstest_amd import codegen, models
  m = models.load(model, disable_contact=True)
  path = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)[0]
  kernels = {}
  for r in csv.DictReader(open(path)):
    name = r["Name"]
    base = name.split("(")[0].replace("void ", "").split("<")[0]
    if base == f"k_all_{model}" or base.startswith("k_constraint"):
      kernels[base] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                       "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3}
  launch_ms = sum(k["avg_us"] for k in kernels.values()) / 1e3
  out = {"model": model, "batch": 65536, "source_sha": codegen.source_hash(m, model),
         "kernels": kernels, "launch_ms": launch_ms, "stats_file": os.path.relpath(path, src),
         "note": "sum of the per-dispatch average durations of the hot-path kernels of one "
                 "launch, from rocprofv3 --kernel-trace --stats over python bench.py"}
  json.dump(out, open(dst, "w"), indent=1)
  print(json.dumps(out, indent=1))


if __name__ == "__main__":
  main(*sys.argv[1:])
