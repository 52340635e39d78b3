"""Summarize tools/pmc.sh output into HBM traffic per hot-path launch (profiles/<round>/).

  python tools/pmc_summary.py gpurun_out profiles/r01/pmc_traffic.json
  python tools/pmc_summary.py gpurun_out profiles/r05/pmc_traffic_c4.json 4 4096

FETCH_SIZE / WRITE_SIZE (KB per dispatch) come from separate rocprofv3 --pmc passes of the
same bench command (tools/pmc.sh). Correction (MI355X_MICROARCH.md, HBM section): on gfx950
FETCH_SIZE reports half the bytes of a coalesced streaming read. The factor is calibrated on
this engine's own access pattern with k_fac, whose reads are exactly qM (nM doubles per
instance). WRITE_SIZE is taken as is and checked the same way against k_pos's known stores.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


# FETCH_SIZE correction for this engine's 8-byte-per-lane mirror reads, calibrated on the
# staged k_fac_humanoid, whose reads are exactly qM (profiles/r01/pmc_v7_pass2.csv: 1.9623)
CALIB_8B = 1.9623055899886392


def per_kernel(path, counter):
  vals = collections.defaultdict(list)
  for r in csv.DictReader(open(path)):
    if r["Counter_Name"] == counter:
      vals[r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]].append(
          float(r["Counter_Value"]) * 1024.0)
  return {k: sum(v) / len(v) for k, v in vals.items()}


def main(src, dst, config=2, batch=65536):
  """config 2: the headline (humanoid, contacts off, batch 65,536); config 4: humanoid with
  contacts (k_all_humanoid_contact + the constraint kernel) at `batch`."""
  from mujoco_inversedynamicstest_amd import models
  contacts = config == 4
  m = models.load("humanoid", disable_contact=not contacts)
  name = "humanoid_contact" if contacts else "humanoid"
  B = batch
  fetch = per_kernel(os.path.join(src, "pmc_2", "pmc_counter_collection.csv"), "FETCH_SIZE")
  write = per_kernel(os.path.join(src, "pmc_3", "pmc_counter_collection.csv"), "WRITE_SIZE")
  if "k_fac_humanoid" in fetch:
    calib = 8.0 * m.nM * B / fetch["k_fac_humanoid"]
  else:   # fused launch: the factor calibrated on the staged k_fac (8-byte lane accesses)
    calib = CALIB_8B
  kernels = [k for k in fetch if k.startswith("k_") and ("humanoid" in k or k.startswith("k_constraint"))]
  if contacts:
    kernels = [k for k in kernels if "contact" in k or k.startswith("k_constraint")]
  else:
    kernels = [k for k in kernels if "contact" not in k]
  rows = {k: {"fetch_bytes": fetch[k] * calib, "write_bytes": write.get(k, 0.0)} for k in kernels}
  total = sum(v["fetch_bytes"] + v["write_bytes"] for v in rows.values())
  from mujoco_inversedynamicstest_amd import codegen
  out = {"batch": B, "model": name, "config": config, "fetch_correction": calib,
         "source_sha": codegen.source_hash(m, name),
         "kernels": rows, "traffic_bytes_per_launch": total,
         "traffic_bytes_per_eval": total / B,
         "note": "FETCH_SIZE x correction (calibrated on k_fac reading exactly qM) + WRITE_SIZE, "
                 "averaged over the dispatches of tools/pmc.sh"}
  json.dump(out, open(dst, "w"), indent=1)
  print(json.dumps(out, indent=1))


if __name__ == "__main__":
  main(sys.argv[1], sys.argv[2], *(int(x) for x in sys.argv[3:5]))
