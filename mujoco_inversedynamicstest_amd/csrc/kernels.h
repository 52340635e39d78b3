// kernels.h -- what the translation units of libmjhip.so share about the big kernels:
// kern_constraint.hip (k_constraint, k_constraint_coop), kern_inverse.hip (k_inverse) define
// and explicitly instantiate them; mjhip.hip launches them (extern template declarations
// below). The split lets the units compile in parallel (__graft_entry__.build()).
#pragma once
#include <hip/hip_runtime.h>

#include "engine_device.h"
#include "post_pass.h"

using mjh::Lane;
using mjh::SP;

//==================================== kernels ===============================================

// Straight-line kernels generated per bundled model by codegen.py (build(), gen_fast.hip),
// selected by model signature (mjhip_fastKernels); each appends limit-active instances to a
// work-list that the constraint kernel then serves.

// generic pipeline over the instances of a work-list (limit-active instances of the fast
// path); grid = ceil(B/64) blocks, threads past *count exit at once
// the fused constraint path's chain masks, one per body, shared by the block (LDS)
#define MJHIP_CHAIN_TABLE(FUSED)                                                         \
  __shared__ unsigned long long chain[64];                                                \
  if (FUSED) {                                                                            \
    if ((int)threadIdx.x < m.nbody) chain[threadIdx.x] = mjh::chainMask(m, threadIdx.x);  \
    __syncthreads();                                                                      \
  }

// fused contact kernels: collision reads geom positions from a per-lane LDS copy (dynamic
// shared memory of mjh::gstageBytes, [3*ngeom][64 lanes])
extern __shared__ double g_gstage[];
#define MJHIP_GEOM_STAGE(C, F)                                                           \
  if (C && F) {                                                                           \
    d.gxpos.p = g_gstage + threadIdx.x;                                                   \
    d.gstage = true;                                                                      \
  }

// Cooperative constraint part (the fused path of k_constraint, G lanes per instance).
//
// One wave holds 64/G instances; the G lanes of an instance's group split its work:
//   collision   the model's static geom-pair program (collisionPairs, host-built in the order
//               the serial mj_collision emits contacts), G pairs per round: each lane counts
//               its pair's contacts, a group prefix sum places them, the lane writes them
//   rows        equality (lane 0), then friction and limit rows: every lane evaluates the
//               predicates (so all agree on the row numbers), the owner of row r (r % G)
//               writes and finishes it; contact rows: contact c belongs to lane c % G, a
//               prefix sum over the contacts' row counts gives each its first row
//   J'force     column-parallel (column j on lane j % G): each column's sum runs over the
//               rows in order, as mju_mulMatTVec's, then the mj_inverse assembly
// Every output equals the serial (one lane per instance) fused path's.
template <int G>
__device__ __forceinline__ int groupScan(int x, int sub, int* total) {
  for (int o = 1; o < G; o <<= 1) {
    const int y = __shfl_up(x, o, G);
    if (sub >= o) x += y;
  }
  *total = __shfl(x, G - 1, G);
  return x;                               // inclusive
}

template <int S>
__device__ __forceinline__ void rowFields(const Lane<S>& d, int r, double pos, double margin,
                                          double frictionloss, int type, int id) {
  d.efc_pos[r] = pos;
  d.efc_margin[r] = margin;
  d.efc_frictionloss[r] = frictionloss;
  d.efc_type[r] = type;
  d.efc_id[r] = id;
}

// grid of k_constraint_coop: one group per instance, or for a work-list (whose length only
// the device knows) at most one block per SIMD striding over it
static unsigned coopGrid(int B, int G, bool list) {
  const unsigned full = (unsigned)((B + 64/G - 1) / (64/G));
  return list && full > 1024u ? 1024u : full;
}

// CoopPair, the pair program entry: engine_device.h (the generic collision() reads it too)

// dynamic LDS of k_constraint_coop: the pair program and geom_size once per block; per
// instance 8 nv
// doubles (cdof, qvel, qacc), qpos, the geom frames (geom_xpos, geom_xmat), the survivor
// list of the sphere filter (npair ints), the bodies of the first kCoopContacts contacts (4
// ints each) and the forces of the first kCoopRows rows (later ones are read back from
// efc_force); with box-box pairs, 72 doubles per lane for their contact positions. The caps
// keep a block small enough that every wave of a 4,096 batch is resident at once (the
// humanoid's worst-case capacities, 273 contacts and 424 rows, would allow two blocks per CU).
constexpr int kBoxBoxBuf = 72;
constexpr int kCoopContacts = 64;
#ifndef MJHIP_COOP_CQ
#define MJHIP_COOP_CQ 2
#endif
constexpr int kCoopContactLanes = MJHIP_COOP_CQ;   // lanes per contact in the contact rows
constexpr int kCoopRows = 128;
__host__ __device__ static inline int coopContacts(int con_cap) {
  return con_cap < kCoopContacts ? con_cap : kCoopContacts;
}
__host__ __device__ static inline int coopRows(int efc_cap) {
  return efc_cap < kCoopRows ? efc_cap : kCoopRows;
}
__host__ __device__ static inline int coopPerInstance(const mjhipModel& m, int npair,
                                                      int con_cap, int efc_cap) {
  return 8*m.nv + m.nq + 12*m.ngeom + (npair + 1) / 2 + 3*coopContacts(con_cap) +
         coopRows(efc_cap);
}
static unsigned coopLdsBytes(const mjhipModel& m, int G, int efc_cap, bool boxpair, int npair,
                             int con_cap) {
  return (unsigned)((kCoopPairDoubles*npair + 3*m.ngeom +
                     (64 / G) * coopPerInstance(m, npair, con_cap, efc_cap) +
                     (boxpair ? 64*kBoxBoxBuf : 0)) * sizeof(double));
}

template <bool CONTACT, bool FUSED, bool LIST>
__global__ __launch_bounds__(64) void k_constraint(mjhipModel m, Mirror mr, int B,
                                                   const int* __restrict__ worklist,
                                                   const int* __restrict__ count,
                                                   double* __restrict__ qfrc_out,
                                                   int* __restrict__ status);
template <int G, bool CONTACT, bool LIST, bool BOX>
__global__ __launch_bounds__(64) void k_constraint_coop(mjhipModel m, Mirror mr, int B,
                                                        const int* __restrict__ worklist,
                                                        const int* __restrict__ count,
                                                        const CoopPair* __restrict__ pairs,
                                                        const mjh::ContactParam* __restrict__ cparams,
                                                        const unsigned long long* __restrict__ masks,
                                                        int npair,
                                                        double* __restrict__ qfrc_out,
                                                        int* __restrict__ status,
                                                        int* __restrict__ cstat);
template <int SKIP, bool CONTACT, bool FUSED>
__global__ __launch_bounds__(64) void k_inverse(mjhipModel m, Mirror mr, int B,
                                                const double* __restrict__ qpos_in,
                                                const double* __restrict__ qvel_in,
                                                const double* __restrict__ qacc_in,
                                                double* __restrict__ qfrc_out,
                                                int* __restrict__ status, int skipsensor);

// mjhip_ccdBatch's kernel (kern_ccd.hip): kCcdOut doubles per pair out (dist, nx, x1[3*50],
// x2[3*50]); nonzero when the launch failed
constexpr long kCcdOut = 2 + 6*mjh::CCD_MAXCON;
int mjhip_launchCcd(hipStream_t s, const mjhipModel& m, int n, const int* g1, const int* g2,
                    const double* in, const double* margin, int N, double tol, int maxc,
                    double cutoff, double* x, int* xi, double* out, int* bad);

// the instantiations libmjhip.so launches (launch_inverse)
#ifndef MJHIP_KERNEL_UNIT
extern template __global__ void k_constraint<true, true, false>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
extern template __global__ void k_constraint<true, false, false>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
extern template __global__ void k_constraint<false, true, false>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
extern template __global__ void k_constraint<false, false, false>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
extern template __global__ void k_constraint<false, true, true>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
extern template __global__ void k_constraint<false, false, true>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
extern template __global__ void k_constraint_coop<16, true, true, true>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
extern template __global__ void k_constraint_coop<16, true, false, true>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
extern template __global__ void k_constraint_coop<16, true, true, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
extern template __global__ void k_constraint_coop<16, true, false, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
extern template __global__ void k_constraint_coop<16, false, true, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
extern template __global__ void k_constraint_coop<16, false, false, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
extern template __global__ void k_inverse<0, true, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
extern template __global__ void k_inverse<0, false, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
extern template __global__ void k_inverse<1, true, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
extern template __global__ void k_inverse<1, false, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
extern template __global__ void k_inverse<2, true, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
extern template __global__ void k_inverse<2, false, false>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
extern template __global__ void k_inverse<0, true, true>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
extern template __global__ void k_inverse<0, false, true>(mjhipModel, Mirror, int, const double*, const double*, const double*, double*, int*, int);
#endif

// each unit's copy of the per-stage timer pointer (engine_device.h mjh_tbuf), set by
// mjhip_contextTimers around a timed call: blocking copies (timed calls are synchronous)
#define MJHIP_TIMER_SETTER(fn)                                                             \
  int fn(unsigned long long* p) {                                                          \
    return hipMemcpyToSymbol(HIP_SYMBOL(mjh_tbuf), &p, sizeof(p)) != hipSuccess;            \
  }
int mjhip_setTimerBufConstraint(unsigned long long* p);   // kern_constraint.hip
int mjhip_setTimerBufInverse(unsigned long long* p);      // kern_inverse.hip
