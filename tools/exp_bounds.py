"""Performance experiment (not part of the product): per-stage bounds of the humanoid kernels.

  python tools/exp_bounds.py          # build tools/exp/libexp.so (here, no GPU needed)
  python tools/exp_bounds.py run      # on the GPU box

For each stage kernel (k_pos, k_fac, k_va) three variants over the same mirror:
  full      the product kernel
  compute   the same code storing only qfrc_inverse (intermediate fields keep the values
            the full run wrote, so later stages read valid data)
  memory    no arithmetic: exactly the stage's mirror loads, then exactly its stores
The inputs are sampled humanoid states (config-2 sampler), batch 65,536, HIP-event timing.
"""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mujoco_inversedynamicstest_amd import codegen, fields, models  # noqa: E402

EXP = os.path.join(ROOT, "tools", "exp")
STAGES = codegen.STAGES


def _stage_io(body):
  """(loads, stores) of a generated stage body: sets of (field, index)."""
  stores = set(re.findall(r"P_(\w+)\[(\d+)\*64\] =", body))
  loads = set(re.findall(r"= P_(\w+)\[(\d+)\*64\]", body)) | set(
      re.findall(r"[-+*] P_(\w+)\[(\d+)\*64\]", body))
  return loads, stores


def _ordered_kernel(st, body, S):
  """The stage's mirror accesses in program order, without the arithmetic."""
  lines = [f"__global__ __launch_bounds__(64, 1) void k_ord_{st}(Mirror mr, int B) {{",
           "  const long blk = blockIdx.x, lane = threadIdx.x;",
           "  double acc = 0.0;"]
  for mm in re.finditer(r"(P_(\w+)\[(\d+)\*64\] =)|(P_(\w+)\[(\d+)\*64\])", body):
    if mm.group(1):
      f, k = mm.group(2), mm.group(3)
      lines.append(f"  mr.{f}[(blk*{S[f]} + {k})*64 + lane] = acc + {k}.0;")
    else:
      f, k = mm.group(5), mm.group(6)
      lines.append(f"  acc += mr.{f}[(blk*{S[f]} + {k})*64 + lane];")
  lines.append("}")
  return "\n".join(lines)


def _memory_kernel(st, loads, stores, S):
  lines = [f"__global__ __launch_bounds__(64, 1) void k_mem_{st}(Mirror mr, int B) {{",
           "  const long blk = blockIdx.x, lane = threadIdx.x;",
           "  double acc = 0.0;"]
  for f, k in sorted(loads, key=lambda x: (x[0], int(x[1]))):
    lines.append(f"  acc += mr.{f}[(blk*{S[f]} + {k})*64 + lane];")
  lines.append("  if (acc == 1.2345e300) acc = 0;   // keep the loads")
  for f, k in sorted(stores, key=lambda x: (x[0], int(x[1]))):
    lines.append(f"  mr.{f}[(blk*{S[f]} + {k})*64 + lane] = acc + {k}.0;")
  lines.append("}")
  return "\n".join(lines)


def build():
  m = models.load("humanoid", disable_contact=True)
  M = codegen._Model(m)
  S = {f.name: f.size(m.sizes) for f in fields.DATA_FIELDS}
  gens = {st: (lambda M, st=st: codegen._GEN[st](M, None)) for st in STAGES}
  full = codegen.generate(m, "full")
  comp = codegen.generate(m, "comp", store_fields={"qfrc_inverse"})
  mem = []
  for st in STAGES:
    body = gens[st](M)
    loads, stores = _stage_io(body)
    mem.append(_memory_kernel(st, loads, stores, S))
    mem.append(_ordered_kernel(st, body, S))
  sizes = ", ".join(f"{k} = {m.sizes.get(k, 0)}" for k in fields.MODEL_SIZES)
  calls = {
      "pos": "mr, B, nullptr, nullptr, nullptr, wl, wc, nullptr, ec",
      "fac": "mr, B, ec", "va": "mr, B, nullptr, nullptr, ec"}
  launch = []
  for v in ("full", "comp"):
    for i, st in enumerate(STAGES):
      launch.append(f"    if (variant == {0 if v == 'full' else 1} && stage == {i}) "
                    f"hipLaunchKernelGGL(k_{st}_{v}, g, b, 0, 0, {calls[st]});")
  for i, st in enumerate(STAGES):
    launch.append(f"    if (variant == 2 && stage == {i}) "
                  f"hipLaunchKernelGGL(k_mem_{st}, g, b, 0, 0, mr, B);")
    launch.append(f"    if (variant == 3 && stage == {i}) "
                  f"hipLaunchKernelGGL(k_ord_{st}, g, b, 0, 0, mr, B);")
  src = f'''#include <hip/hip_runtime.h>
#include <string.h>
#include "{ROOT}/mujoco_inversedynamicstest_amd/csrc/engine_device.h"
{full}
{comp}
{chr(10).join(mem)}
static Mirror mr;
static int *wl, *wc, *ec;
static int Bcap = 0;
extern "C" int setup(int B, const double* qpos, const double* qvel, const double* qacc) {{
  memset(&mr, 0, sizeof(mr));
  const int nblk = (B + 63) / 64;
#define MJ_M(n) n
  int {sizes};
#define XD(name, d0, d1, stage) mr.name##_n = (d0) * (d1); \\
  if (hipMalloc((void**)&mr.name, sizeof(double) * (size_t)nblk * 64 * (mr.name##_n + 1))) \\
    return 1; \\
  hipMemset(mr.name, 0, sizeof(double) * (size_t)nblk * 64 * (mr.name##_n + 1));
  MJHIP_DATA_FIELDS
#undef XD
  hipMemcpy(mr.qpos, qpos, sizeof(double) * (size_t)nblk * 64 * nq, hipMemcpyHostToDevice);
  hipMemcpy(mr.qvel, qvel, sizeof(double) * (size_t)nblk * 64 * nv, hipMemcpyHostToDevice);
  hipMemcpy(mr.qacc, qacc, sizeof(double) * (size_t)nblk * 64 * nv, hipMemcpyHostToDevice);
  hipMalloc((void**)&wl, sizeof(int) * (B + 1)); hipMalloc((void**)&wc, 4);
  hipMalloc((void**)&ec, sizeof(int) * 4 * (size_t)nblk * 64);
  hipMemset(ec, 0, sizeof(int) * 4 * (size_t)nblk * 64);
  Bcap = B;
  return hipDeviceSynchronize() != hipSuccess;
}}
// average ms of one launch of (variant, stage)
extern "C" float run(int variant, int stage, int reps) {{
  const int B = Bcap, nblk = (B + 63) / 64;
  dim3 g(nblk), b(64);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int r = -2; r < reps; r++) {{
    if (r == 0) hipEventRecord(e0);
    hipMemset(wc, 0, 4);
{chr(10).join(launch)}
  }}
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}}
extern "C" int worklist() {{ int n; hipMemcpy(&n, wc, 4, hipMemcpyDeviceToHost); return n; }}
'''
  os.makedirs(EXP, exist_ok=True)
  p = os.path.join(EXP, "exp.hip")
  open(p, "w").write(src)
  subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                  "-shared", "-Wno-unused-value", "-o", os.path.join(EXP, "libexp.so"), p],
                 check=True)
  io = {}
  for st in STAGES:
    loads, stores = _stage_io(gens[st](M))
    io[st] = (len(loads), len(stores))
  open(os.path.join(EXP, "io.txt"), "w").write(repr(io))


def _mirror(x, B):
  """Row-major (B, n) -> mirror layout [blk][k][64]."""
  n = x.shape[1]
  return np.ascontiguousarray(x.reshape(B // 64, 64, n).transpose(0, 2, 1))


def run():
  import torch  # noqa: F401  (one HIP runtime per process)
  from mujoco_inversedynamicstest_amd.sampler import sample_states
  L = ctypes.CDLL(os.path.join(EXP, "libexp.so"))
  L.run.restype = ctypes.c_float
  L.run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
  L.setup.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3
  io = eval(open(os.path.join(EXP, "io.txt")).read())
  m = models.load("humanoid", disable_contact=True)
  B = 65536
  q, v, a = sample_states(m, B)
  q, v, a = _mirror(q, B), _mirror(v, B), _mirror(a, B)
  assert L.setup(B, q.ctypes.data, v.ctypes.data, a.ctypes.data) == 0
  print(f"{'stage':6s} {'loads':>6s} {'stores':>6s} {'full us':>9s} {'compute us':>11s} "
        f"{'memory us':>10s} {'mem TB/s':>9s} {'ordered us':>10s}", flush=True)
  tot = [0.0, 0.0, 0.0, 0.0]
  for i, st in enumerate(STAGES):
    t = [L.run(var, i, 20) * 1e3 for var in (0, 1, 2, 3)]
    if i == 0:
      t[0] = L.run(0, 0, 20) * 1e3   # full first so intermediate fields are valid
    nl, ns = io[st]
    tb = (nl + ns) * 8 * B / (t[2] * 1e-6) / 1e12
    for k in range(4):
      tot[k] += t[k]
    print(f"{st:6s} {nl:6d} {ns:6d} {t[0]:9.1f} {t[1]:11.1f} {t[2]:10.1f} {tb:9.2f} "
          f"{t[3]:10.1f}", flush=True)
  print(f"{'total':20s} {tot[0]:9.1f} {tot[1]:11.1f} {tot[2]:10.1f} {'':9s} {tot[3]:10.1f}"
        f"   worklist={L.worklist()}")


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "run":
    run()
  else:
    build()
