"""Performance experiment (not part of the product): HBM write rate vs store width / hint.

  python tools/exp_stores.py        # build tools/exp/libstores.so
  python tools/exp_stores.py run    # GPU box

Each kernel writes N doubles per lane for a 65,536-lane grid (64-lane blocks, one wave per
SIMD, like the engine). Variants: 8-byte stores ([k][64] layout, the current mirror),
16-byte stores ([k/2][64][2] layout), each plain and non-temporal.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXP = os.path.join(ROOT, "tools", "exp")
N = 1790

SRC = r'''
#include <hip/hip_runtime.h>
#define N %(N)d
__global__ __launch_bounds__(64, 1) void k_st8(double* out) {
  double* p = out + (long)blockIdx.x * N * 64 + threadIdx.x;
  double v = threadIdx.x;
#pragma unroll 16
  for (int k = 0; k < N; k++) p[k * 64] = v + k;
}
__global__ __launch_bounds__(64, 1) void k_st8nt(double* out) {
  double* p = out + (long)blockIdx.x * N * 64 + threadIdx.x;
  double v = threadIdx.x;
#pragma unroll 16
  for (int k = 0; k < N; k++) __builtin_nontemporal_store(v + k, p + k * 64);
}
__global__ __launch_bounds__(64, 1) void k_st16(double* out) {
  double2* p = (double2*)(out + (long)blockIdx.x * N * 64) + threadIdx.x;
  double v = threadIdx.x;
#pragma unroll 16
  for (int k = 0; k < N / 2; k++) p[k * 64] = make_double2(v + 2 * k, v + 2 * k + 1);
}
__global__ __launch_bounds__(64, 1) void k_st16nt(double* out) {
  double2* p = (double2*)(out + (long)blockIdx.x * N * 64) + threadIdx.x;
  double v = threadIdx.x;
#pragma unroll 16
  for (int k = 0; k < N / 2; k++) {
    double2 x = make_double2(v + 2 * k, v + 2 * k + 1);
    __builtin_nontemporal_store(x.x, &p[k * 64].x);
    __builtin_nontemporal_store(x.y, &p[k * 64].y);
  }
}
static double* buf = nullptr;
extern "C" float run(int which, int lanes, int reps) {
  const int nblk = lanes / 64;
  if (!buf && hipMalloc((void**)&buf, sizeof(double) * (size_t)lanes * N)) return -1;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int r = -2; r < reps; r++) {
    if (r == 0) hipEventRecord(e0);
    if (which == 0) hipLaunchKernelGGL(k_st8, dim3(nblk), dim3(64), 0, 0, buf);
    if (which == 1) hipLaunchKernelGGL(k_st8nt, dim3(nblk), dim3(64), 0, 0, buf);
    if (which == 2) hipLaunchKernelGGL(k_st16, dim3(nblk), dim3(64), 0, 0, buf);
    if (which == 3) hipLaunchKernelGGL(k_st16nt, dim3(nblk), dim3(64), 0, 0, buf);
  }
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}
'''


def build():
  os.makedirs(EXP, exist_ok=True)
  p = os.path.join(EXP, "stores.hip")
  open(p, "w").write(SRC % {"N": N})
  subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                  "-o", os.path.join(EXP, "libstores.so"), p], check=True)


def run():
  L = ctypes.CDLL(os.path.join(EXP, "libstores.so"))
  L.run.restype = ctypes.c_float
  L.run.argtypes = [ctypes.c_int] * 3
  lanes = 65536
  for w, name in enumerate(("8B", "8B nt", "16B", "16B nt")):
    ms = L.run(w, lanes, 20)
    print(f"{name:7s} {ms*1e3:8.1f} us  {8*N*lanes/ms/1e9:7.0f} GB/s", flush=True)


if __name__ == "__main__":
  run() if len(sys.argv) > 1 and sys.argv[1] == "run" else build()
