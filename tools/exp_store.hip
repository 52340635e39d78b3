// Performance experiment (not part of the product): store throughput of one wave per SIMD
// for the mirror layouts. Each lane writes N doubles, as k_all's stage stores do:
//   layout 0  [k][64 lanes]          one dwordx2 per lane per component (the mirror today)
//   layout 1  [k/2][64 lanes][2]     two components per lane adjacent: dwordx4 stores
// Occupancy is pinned with dynamic LDS (waves per SIMD = 160 KB / 4 / lds), streaming
// (non-temporal) or plain stores. Build: hipcc --offload-arch=gfx950 -O3 -o exp_store
// tools/exp_store.hip; run: ./exp_store
#include <hip/hip_runtime.h>

#include <stdio.h>

constexpr int N = 2560;                 // doubles per instance (20 KB, k_all's B_eval)

template <int LAYOUT, bool NT>
__global__ __launch_bounds__(64) void k_store(double* __restrict__ out, double seed) {
  extern __shared__ double lds[];
  const long blk = blockIdx.x;
  const int lane = threadIdx.x;
  double x = seed + lane;
  if (seed < 0) lds[lane] = x;          // keeps the LDS allocation (never true)
  double* base = out + blk * (long)N * 64;
#pragma unroll 16
  for (int k = 0; k < N; k += 2) {
    const double a = x * 1.0000001 + k, b = x * 0.9999999 - k;
    if (LAYOUT == 0) {
      if (NT) {
        __builtin_nontemporal_store(a, base + (long)k * 64 + lane);
        __builtin_nontemporal_store(b, base + (long)(k + 1) * 64 + lane);
      } else {
        base[(long)k * 64 + lane] = a;
        base[(long)(k + 1) * 64 + lane] = b;
      }
    } else {
      double2* p = reinterpret_cast<double2*>(base + (long)(k / 2) * 128 + 2 * lane);
      if (NT) {
        __builtin_nontemporal_store(a, &p->x);
        __builtin_nontemporal_store(b, &p->y);
      } else {
        *p = make_double2(a, b);
      }
    }
    x = x * 1.0000001;
  }
}

template <int LAYOUT, bool NT>
static float run(double* out, int blocks, int lds, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_store<LAYOUT, NT>), dim3(blocks), dim3(64), lds, 0, out, 1.0);
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; r++) {
    hipLaunchKernelGGL((k_store<LAYOUT, NT>), dim3(blocks), dim3(64), lds, 0, out, 1.0);
  }
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const int blocks = 1024;              // 65,536 instances
  double* out = nullptr;
  const size_t bytes = (size_t)blocks * N * 64 * sizeof(double);
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  printf("%zu bytes per launch\n", bytes);
  for (int wps : {1, 2, 4}) {
    const int lds = 160 * 1024 / 4 / wps - 1024;
    float t00 = run<0, false>(out, blocks, lds, 10), t01 = run<0, true>(out, blocks, lds, 10);
    float t10 = run<1, false>(out, blocks, lds, 10), t11 = run<1, true>(out, blocks, lds, 10);
    printf("waves/SIMD %d: [k][64] plain %.1f us %.2f TB/s, NT %.1f us %.2f TB/s; "
           "[k/2][64][2] plain %.1f us %.2f TB/s, NT %.1f us %.2f TB/s\n", wps,
           t00 * 1e3, bytes / t00 / 1e9, t01 * 1e3, bytes / t01 / 1e9,
           t10 * 1e3, bytes / t10 / 1e9, t11 * 1e3, bytes / t11 / 1e9);
  }
  hipFree(out);
  return 0;
}
