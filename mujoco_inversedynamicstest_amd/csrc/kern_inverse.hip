// kern_inverse.hip -- the generic fused mj_inverseSkip kernel k_inverse (every skipstage,
// with and without contacts), in its own translation unit of libmjhip.so (kernels.h).
#define MJHIP_KERNEL_UNIT 1
#include "kernels.h"

// Fused mj_inverseSkip over a batch. Optional row-major (instance-major) inputs are copied
// into the mirror first; optional row-major qfrc_inverse output is written at the end.
template <int SKIP, bool CONTACT, bool FUSED>
__global__ __launch_bounds__(64) void k_inverse(mjhipModel m, Mirror mr, int B,
                                                const double* __restrict__ qpos_in,
                                                const double* __restrict__ qvel_in,
                                                const double* __restrict__ qacc_in,
                                                double* __restrict__ qfrc_out,
                                                int* __restrict__ status, int skipsensor) {
  MJHIP_CHAIN_TABLE(FUSED)
  const int blk = blockIdx.x, lane = threadIdx.x;
  const long inst = (long)blk*64 + lane;
  if (inst >= B) return;
  Lane<64> d = lane_view(mr, blk, lane);
  d.chain = chain;
  MJHIP_GEOM_STAGE(CONTACT, FUSED)
  if (qpos_in) {
    for (int k = 0; k < m.nq; k++) d.qpos[k] = qpos_in[inst*m.nq + k];
  }
  if (qvel_in) {
    for (int k = 0; k < m.nv; k++) d.qvel[k] = qvel_in[inst*m.nv + k];
  }
  if (qacc_in) {
    for (int k = 0; k < m.nv; k++) d.qacc[k] = qacc_in[inst*m.nv + k];
  }
  MJH_PHASE0(0, 24);
  int st = mjh::inverseSkip<64, CONTACT, FUSED>(m, d, SKIP, skipsensor);
  if (qfrc_out) {
    for (int k = 0; k < m.nv; k++) qfrc_out[inst*m.nv + k] = d.qfrc_inverse[k];
  }
  if (status) status[inst] = st;
}

template __global__ void k_inverse<0, true, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
template __global__ void k_inverse<0, false, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
template __global__ void k_inverse<1, true, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
template __global__ void k_inverse<1, false, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
template __global__ void k_inverse<2, true, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
template __global__ void k_inverse<2, false, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
template __global__ void k_inverse<0, true, true>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
template __global__ void k_inverse<0, false, true>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);

MJHIP_TIMER_SETTER(mjhip_setTimerBufInverse)
