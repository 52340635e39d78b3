"""Performance experiment (not part of the product): bounds of the humanoid fast kernel.

Builds tools/exp/libexp.so with three kernels over the same mirror layout:
  full      the product straight-line kernel (all 2,563 doubles stored)
  qfrc      the same code storing only qfrc_inverse
  stores    no compute: every lane writes all 2,563 output doubles (write roofline)
and times each at batch 65,536 with HIP events (run on the GPU box).
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mujoco_inversedynamicstest_amd import codegen, fields, models  # noqa: E402

EXP = os.path.join(ROOT, "tools", "exp")


def build():
  m = models.load("humanoid", disable_contact=True)
  full = codegen.generate(m, "full")
  qfrc = codegen.generate(m, "qfrc", store_fields={"qfrc_inverse"})
  S = {f.name: f.size(m.sizes) for f in fields.DATA_FIELDS if f.stage > 0}
  stores = ["__global__ __launch_bounds__(64, 1) void k_stores(Mirror mr, int B) {",
            "  const int blk = blockIdx.x, lane = threadIdx.x;",
            "  double v = (double)lane;"]
  for name, n in S.items():
    if n:
      stores.append(f"  {{ double* p = mr.{name} + ((long)blk*{n})*64 + lane;"
                    f" for (int k = 0; k < {n}; k++) p[k*64] = v + k; }}")
  stores.append("}")
  src = f'''#include <hip/hip_runtime.h>
#include <string.h>
#include "{ROOT}/mujoco_inversedynamicstest_amd/csrc/engine_device.h"
{full}
{qfrc}
{chr(10).join(stores)}
extern "C" float run(int which, int B, int reps) {{
  Mirror mr; memset(&mr, 0, sizeof(mr));
  const int nblk = (B + 63) / 64;
#define MJ_M(n) n
  int nq = 28, nv = 27, nbody = 17, njnt = 22, ngeom = 20, nsite = 0, ncam = 3, nlight = 2,
      ntendon = 2, nu = 21, nJmom = 21, nM = 243, nC = 243;
  (void)nsite;
#define XD(name, d0, d1, stage) mr.name##_n = (d0) * (d1); \\
  hipMalloc((void**)&mr.name, sizeof(double) * (size_t)nblk * 64 * (mr.name##_n + 1)); \\
  hipMemset(mr.name, 0, sizeof(double) * (size_t)nblk * 64 * (mr.name##_n + 1));
  MJHIP_DATA_FIELDS
#undef XD
  int *wl, *wc, *ec;
  hipMalloc((void**)&wl, sizeof(int) * (B + 1)); hipMalloc((void**)&wc, 4);
  hipMalloc((void**)&ec, sizeof(int) * 4 * (size_t)nblk * 64);
  // plausible states: qpos0-like quaternion
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  dim3 g(nblk), b(64);
  for (int r = -2; r < reps; r++) {{
    if (r == 0) hipEventRecord(e0);
    hipMemset(wc, 0, 4);
    if (which == 0) hipLaunchKernelGGL(k_fast_full, g, b, 0, 0, mr, B, nullptr, nullptr,
                                       nullptr, nullptr, nullptr, wl, wc, ec);
    if (which == 1) hipLaunchKernelGGL(k_fast_qfrc, g, b, 0, 0, mr, B, nullptr, nullptr,
                                       nullptr, nullptr, nullptr, wl, wc, ec);
    if (which == 2) hipLaunchKernelGGL(k_stores, g, b, 0, 0, mr, B);
  }}
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}}
'''
  os.makedirs(EXP, exist_ok=True)
  p = os.path.join(EXP, "exp.hip")
  open(p, "w").write(src)
  subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                  "-shared", "-o", os.path.join(EXP, "libexp.so"), p], check=True)


def run():
  import torch  # noqa: F401  (one HIP runtime per process)
  L = ctypes.CDLL(os.path.join(EXP, "libexp.so"))
  L.run.restype = ctypes.c_float
  L.run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
  B = 65536
  bytes_out = 8 * 2563 * B
  for which, name in ((0, "full"), (1, "qfrc_only"), (2, "stores_only")):
    ms = L.run(which, B, 20)
    print(f"{name:12s} {ms*1e3:9.1f} us   {B/ms/1e3:8.2f} Mevals/s   "
          f"{bytes_out/ms/1e6 if which != 1 else 0:8.1f} GB/s(out)", flush=True)


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "run":
    run()
  else:
    build()
