"""Performance experiment (not part of the product): does splitting one instance over L lanes
(L waves per SIMD at batch 65,536) raise the mirror stream rate of k_all_humanoid?

  python tools/exp_occupancy.py          # build tools/exp/libocc.so (here, no GPU needed)
  python tools/exp_occupancy.py run      # on the GPU box

Memory-only twins of the fused kernel: exactly its mirror loads and stores in program order
(the three stage bodies of codegen), no arithmetic. Variant L deals the access list over the
L lanes of an instance round-robin (instruction t of lane h touches access L*t + h, a
per-lane address select), so a wave holds 64/L instances and the grid has 1024*L waves.
"""
import ctypes
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mujoco_inversedynamicstest_amd import codegen, fields, models  # noqa: E402

EXP = os.environ.get("EXP_DIR", os.path.join(ROOT, "tools", "exp"))
LANES = (1, 2, 4)


def accesses():
  m = models.load("humanoid", disable_contact=True)
  M = codegen._Model(m)
  S = {f.name: f.size(m.sizes) for f in fields.DATA_FIELDS}
  acc = []
  for st in codegen.STAGES:
    body = codegen._GEN[st](M, None)
    for mm in re.finditer(r"(P_(\w+)\[(\d+)\*64\] =)|(P_(\w+)\[(\d+)\*64\])", body):
      if mm.group(1):
        acc.append(("st", mm.group(2), int(mm.group(3))))
      else:
        acc.append(("ld", mm.group(5), int(mm.group(6))))
  return S, acc


def kernel(L, S, acc, base):
  lines = [f"__global__ __launch_bounds__(64) void k_occ{L}(double* __restrict__ buf, int B) {{",
           f"  const int h = threadIdx.x & {L - 1};",
           f"  const long blk = blockIdx.x / {L};   // wave-uniform: 64/L instances of one block",
           f"  const long li = (blockIdx.x % {L})*{64 // L} + threadIdx.x / {L};",
           "  double a = 0.0;"]
  # group consecutive accesses of one kind into L-wide instructions
  i = 0
  while i < len(acc):
    kind = acc[i][0]
    grp = [acc[i]]
    while len(grp) < L and i + len(grp) < len(acc) and acc[i + len(grp)][0] == kind:
      grp.append(acc[i + len(grp)])
    i += len(grp)
    offs = [f"({base[f]}L + (blk*{S[f]} + {k})*64)" for _, f, k in grp]
    sel = offs[-1]
    for j in range(len(offs) - 2, -1, -1):
      sel = f"(h == {j} ? {offs[j]} : {sel})"
    if len(grp) < L:          # a short group: the lanes without an access repeat the last one
      pass
    if kind == "st":
      lines.append(f"  buf[{sel} + li] = (double)(h + {i});")
    else:
      lines.append(f"  a += buf[{sel} + li];")
  lines.append("  if (a == 1.2345e300) buf[li] = a;")
  lines.append("}")
  return "\n".join(lines)


def build():
  S, acc = accesses()
  B = 65536
  base, tot = {}, 0
  for f in S:
    base[f] = tot
    tot += B * max(S[f], 1)
  kernels = "\n".join(kernel(L, S, acc, base) for L in LANES)
  launches = "\n".join(
      f"    if (L == {L}) hipLaunchKernelGGL(k_occ{L}, dim3(1024*{L}), dim3(64), 0, 0, buf, B);"
      for L in LANES)
  src = f'''#include <hip/hip_runtime.h>
{kernels}
static double* buf;
extern "C" int setup() {{
  if (hipMalloc((void**)&buf, sizeof(double) * {tot}L)) return 1;
  return hipMemset(buf, 0, sizeof(double) * {tot}L) != hipSuccess;
}}
extern "C" float run(int L, int reps) {{
  const int B = {B};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int r = -2; r < reps; r++) {{
    if (r == 0) hipEventRecord(e0);
{launches}
  }}
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}}
'''
  os.makedirs(EXP, exist_ok=True)
  p = os.path.join(EXP, "occ.hip")
  open(p, "w").write(src)
  subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                  "-shared", "-o", os.path.join(EXP, "libocc.so"), p], check=True)
  nst = sum(1 for a in acc if a[0] == "st")
  open(os.path.join(EXP, "occ.txt"), "w").write(repr((len(acc) - nst, nst)))


def run():
  import torch  # noqa: F401
  L_ = ctypes.CDLL(os.path.join(EXP, "libocc.so"))
  L_.run.restype = ctypes.c_float
  L_.run.argtypes = [ctypes.c_int, ctypes.c_int]
  assert L_.setup() == 0
  nld, nst = eval(open(os.path.join(EXP, "occ.txt")).read())
  print(f"accesses per instance: {nld} loads, {nst} stores", flush=True)
  for L in LANES:
    t = L_.run(L, 20)
    tb = (nld + nst) * 8 * 65536 / (t * 1e-3) / 1e12
    print(f"lanes/instance {L}: {t * 1e3:8.1f} us  {tb:5.2f} TB/s", flush=True)


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "run":
    run()
  else:
    build()
