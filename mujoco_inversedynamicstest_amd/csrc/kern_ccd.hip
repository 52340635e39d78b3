// kern_ccd.hip -- mjhip_ccdBatch's kernel: the native GJK/EPA solver (mjc_ccd) with its box
// multicontact on caller-given frames, in its own translation unit of libmjhip.so
// (kernels.h), compiled without multiply-add contraction (__graft_entry__.UNIT_FLAGS) as the
// oracle is.
#define MJHIP_KERNEL_UNIT 1
#include "kernels.h"

// mjhip_ccdBatch: mjc_ccd on pair i's geoms at its frames (in: 24 doubles per pair, pos1,
// mat1, pos2, mat2; out: kCcdOut per pair, dist, nx, x1[3 mjMAXCONPAIR], x2[...]), scratch
// contiguous per pair; bad[i]: 1 polytope capacity, 2 multicontact outside the subset
__global__ __launch_bounds__(64) void k_ccd(mjhipModel m, int n, const int* __restrict__ g1,
                                            const int* __restrict__ g2,
                                            const double* __restrict__ in,
                                            const double* __restrict__ margin, int N,
                                            double tol, int maxc, double cutoff,
                                            double* __restrict__ x, int* __restrict__ xi,
                                            double* __restrict__ out, int* __restrict__ bad) {
  const int i = blockIdx.x*64 + threadIdx.x;
  if (i >= n) return;
  const double* f = in + 24L*i;
  bad[i] = mjh::ccdGeneral<true>(m, g1[i], g2[i], f, f + 3, f + 12, f + 15,
                                 margin ? margin[i] : 0.0, N, tol, maxc, cutoff,
                                 x + (long)i*mjh::ccdScratchDoubles(N),
                                 xi + (long)i*mjh::ccdScratchInts(N), out + kCcdOut*i);
}


int mjhip_launchCcd(hipStream_t s, const mjhipModel& m, int n, const int* g1, const int* g2,
                    const double* in, const double* margin, int N, double tol, int maxc,
                    double cutoff, double* x, int* xi, double* out, int* bad) {
  hipLaunchKernelGGL(k_ccd, dim3((n + 63)/64), dim3(64), 0, s, m, n, g1, g2, in, margin, N, tol,
                     maxc, cutoff, x, xi, out, bad);
  return hipGetLastError() != hipSuccess;
}
