"""Performance experiment (not part of the product): time generator variants side by side.

  python tools/exp_variants.py            # build tools/exp/libvariants.so (no GPU needed)
  python tools/exp_variants.py run        # GPU box

Each variant is the humanoid's stage kernels generated with different codegen settings
(VARIANTS below). The kernels share one mirror filled with sampled states; a variant's
stages run in pipeline order, timed per stage with HIP events (batch 65,536). Runs of
different variants alternate, so the comparison does not favour a warm cache.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mujoco_inversedynamicstest_amd import codegen, fields, models  # noqa: E402

EXP = os.path.join(ROOT, "tools", "exp")
VARIANTS = {"staged": {}, "half_pos": {"LANES": {"pos": 32, "fac": 64, "va": 64}},
            "half_all": {"LANES": {"pos": 32, "fac": 32, "va": 32}}}


def build():
  m = models.load("humanoid", disable_contact=True)
  srcs, launch = [], []
  for vi, (name, settings) in enumerate(VARIANTS.items()):
    saved = {k: getattr(codegen, k) for k in settings}
    for k, v in settings.items():
      setattr(codegen, k, v)
    srcs.append(codegen.generate(m, name))
    for k, v in saved.items():
      setattr(codegen, k, v)
    calls = {"pos": "mr, B, nullptr, nullptr, nullptr, wl, wc, nullptr, ec",
             "fac": "mr, B, ec", "va": "mr, B, nullptr, nullptr, ec"}
    if settings.get("FUSE"):
      launch.append(f"    if (variant == {vi} && stage == 0) hipLaunchKernelGGL(k_all_{name}, g, b, 0, 0, "
                    "mr, B, nullptr, nullptr, nullptr, nullptr, nullptr, wl, wc, nullptr, ec);")
      continue
    for si, st in enumerate(codegen.STAGES):
      nl = settings.get("LANES", codegen.LANES)[st]
      gb = "g, b" if nl == 64 else f"dim3(g.x*{64 // nl}), dim3({nl})"
      launch.append(f"    if (variant == {vi} && stage == {si}) "
                    f"hipLaunchKernelGGL(k_{st}_{name}, {gb}, 0, 0, {calls[st]});")
  sizes = ", ".join(f"{k} = {m.sizes.get(k, 0)}" for k in fields.MODEL_SIZES)
  src = f'''#include <hip/hip_runtime.h>
#include <string.h>
#include "{ROOT}/mujoco_inversedynamicstest_amd/csrc/engine_device.h"
{chr(10).join(srcs)}
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
// one pipeline pass of `variant`; per-stage ms into ms[]
extern "C" void run(int variant, int nstage, float* ms) {{
  const int B = Bcap, nblk = (B + 63) / 64;
  dim3 g(nblk), b(64);
  hipEvent_t ev[8];
  for (int i = 0; i <= nstage; i++) hipEventCreate(&ev[i]);
  hipMemset(wc, 0, 4);
  hipEventRecord(ev[0]);
  for (int stage = 0; stage < nstage; stage++) {{
{chr(10).join(launch)}
    hipEventRecord(ev[stage + 1]);
  }}
  hipEventSynchronize(ev[nstage]);
  for (int i = 0; i < nstage; i++) hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]);
  for (int i = 0; i <= nstage; i++) hipEventDestroy(ev[i]);
}}
'''
  os.makedirs(EXP, exist_ok=True)
  p = os.path.join(EXP, "variants.hip")
  open(p, "w").write(src)
  subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                  "-shared", "-Wno-unused-value", "-Wno-unused-result", "-o",
                  os.path.join(EXP, "libvariants.so"), p], check=True)


def run(reps=20):
  import numpy as np
  import torch  # noqa: F401  (one HIP runtime per process)
  from mujoco_inversedynamicstest_amd.sampler import sample_states
  L = ctypes.CDLL(os.path.join(EXP, "libvariants.so"))
  L.setup.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3
  L.run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
  m = models.load("humanoid", disable_contact=True)
  B = 65536
  q, v, a = sample_states(m, B)
  mir = lambda x: np.ascontiguousarray(x.reshape(B // 64, 64, -1).transpose(0, 2, 1))
  q, v, a = mir(q), mir(v), mir(a)
  assert L.setup(B, q.ctypes.data, v.ctypes.data, a.ctypes.data) == 0
  ns = len(codegen.STAGES)
  acc = {n: np.zeros(ns) for n in VARIANTS}
  ms = (ctypes.c_float * ns)()
  for r in range(reps + 2):
    for vi, name in enumerate(VARIANTS):
      L.run(vi, ns, ms)
      if r >= 2:
        acc[name] += np.array(ms[:ns])
  for name in VARIANTS:
    t = acc[name] / reps * 1e3
    print(f"{name:8s} " + " ".join(f"{st} {x:7.1f}us" for st, x in zip(codegen.STAGES, t)) +
          f"  total {t.sum():7.1f}us", flush=True)


if __name__ == "__main__":
  run() if len(sys.argv) > 1 and sys.argv[1] == "run" else build()
