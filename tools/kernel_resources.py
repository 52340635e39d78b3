"""Register / scratch usage of the generated kernels for one bundled model (no GPU needed).

  python tools/kernel_resources.py [model]

Compiles only the generated stage kernels for gfx950 with -Rpass-analysis and prints VGPR,
AGPR and scratch bytes per lane for each. Scratch traffic is the thing to drive to zero:
every reload after a mirror store waits for that store (fast path).
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mujoco_inversedynamicstest_amd import codegen, models  # noqa: E402


def resources(name="humanoid", src=None):
  m = models.load(name, disable_contact=True)
  src = src or codegen.generate(m, name)
  with tempfile.TemporaryDirectory() as d:
    hip = os.path.join(d, "k.hip")
    open(hip, "w").write('#include <hip/hip_runtime.h>\n'
                         f'#include "{ROOT}/mujoco_inversedynamicstest_amd/csrc/engine_device.h"\n'
                         + src)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-c", "--offload-device-only", "-Rpass-analysis=kernel-resource-usage",
                        "-Wno-unused-value", "-Wno-unused-result", "-o",
                        os.path.join(d, "k.o"), hip], capture_output=True, text=True)
    if r.returncode:
      raise RuntimeError(r.stderr[-4000:])
  out, cur = {}, None
  for line in r.stderr.splitlines():
    mm = re.search(r"Function Name: _Z\d+(k_\w+?)6Mirror", line)
    if mm:
      cur = mm.group(1)
      out[cur] = {}
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]"):
      mm = re.search(key + r": (\d+)", line)
      if mm and cur:
        out[cur][key.split()[0]] = int(mm.group(1))
  return out


if __name__ == "__main__":
  res = resources(sys.argv[1] if len(sys.argv) > 1 else "humanoid")
  for k, v in res.items():
    print(f"{k:24s} VGPR {v.get('VGPRs')} AGPR {v.get('AGPRs')} scratch {v.get('ScratchSize')} B/lane")
