// mjhip.hip — libmjhip.so: HIP kernels for gfx950 + the C-ABI of include/mjhip.h.
//
// Device layout (DESIGN.md §Data layout):
//   * model: every mjhipModel array copied once into one device buffer; a device-side
//     mjhipModel (same struct, device pointers) is passed by value as a kernel argument, so
//     model reads are wave-uniform scalar loads.
//   * mirror: every per-instance field F of S doubles is F[(blk*S + k)*64 + lane] — 64-
//     instance blocks = one wavefront; a wavefront's access to component k is one 512-byte
//     contiguous segment (fully coalesced), and a block's whole field is contiguous.
//   * one lane per instance (north star), blockDim = 64, grid = ceil(B/64).
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "engine_device.h"
#include "fast_kernels.h"
#include "kernels.h"
#include "pair_program.h"
// lane-count variants of the cooperative kernel (kern_constraint.hip), measurement only
extern template __global__ void k_constraint_coop<8, true, false, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
extern template __global__ void k_constraint_coop<32, true, false, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
#include "post_pass.h"

//==================================== kernels ===============================================

// k_constraint, k_constraint_coop (kern_constraint.hip) and k_inverse (kern_inverse.hip):
// kernels.h

// fluid forces after the generated kernels (csrc/post_pass.h): one lane per instance
__global__ __launch_bounds__(64) void k_fluid_after(mjhipModel m, Mirror mr, int B) {
  const long inst = (long)blockIdx.x*64 + threadIdx.x;
  if (inst >= B) return;
  Lane<64> d = lane_view(mr, blockIdx.x, threadIdx.x);
  mjh::fluidAfter(m, d);
}

// spatial tendons, their transmissions and mj_passive after the generated kernels
// (csrc/post_pass.h): one lane per instance
__global__ __launch_bounds__(64) void k_tendon_after(mjhipModel m, Mirror mr, int B) {
  const long inst = (long)blockIdx.x*64 + threadIdx.x;
  if (inst >= B) return;
  Lane<64> d = lane_view(mr, blockIdx.x, threadIdx.x);
  mjh::tendonAfter(m, d);
}

// mjENBL_INVDISCRETE on the straight-line path (csrc/post_pass.h): mj_discreteAcc and the
// RNE over its qacc before the constraint kernel; the caller's qacc back after the sensors.
// trn: the slider-crank and site transmissions the generated kernels leave to the pass after
// the constraint kernel are formed here first (mj_discreteAcc's implicit damping reads their
// actuator_moment; the reference has them from mj_fwdPosition, before mj_discreteAcc)
__global__ __launch_bounds__(64) void k_discrete_before(mjhipModel m, Mirror mr, int B,
                                                        int trn) {
  const long inst = (long)blockIdx.x*64 + threadIdx.x;
  if (inst >= B) return;
  Lane<64> d = lane_view(mr, blockIdx.x, threadIdx.x);
  if (trn) mjh::transmissionAfter(m, d);
  mjh::discreteBefore(m, d);
}

__global__ __launch_bounds__(64) void k_discrete_restore(mjhipModel m, Mirror mr, int B) {
  const long inst = (long)blockIdx.x*64 + threadIdx.x;
  if (inst >= B) return;
  Lane<64> d = lane_view(mr, blockIdx.x, threadIdx.x);
  mjh::discreteRestore(m, d);
}

// Status checks of the straight-line path: mj_checkPos/Vel/Acc (engine_forward.c:53-102)
// on the inputs and the pivot test behind MJHIP_INST_INERTIA on qLD's diagonal, ORed into
// the status words the generated kernels and k_constraint wrote. A separate launch, run
// only when statuses are asked for: inside the generated kernels the extra live values
// cost spills (tools/kernel_resources.py).
__global__ __launch_bounds__(64) void k_check(mjhipModel m, Mirror mr, int B,
                                              int* __restrict__ status, int skipstage) {
  const long inst = (long)blockIdx.x*64 + threadIdx.x;
  if (inst >= B) return;
  Lane<64> d = lane_view(mr, blockIdx.x, threadIdx.x);
  int st = mjh::checkInputs(m, d, skipstage);
  for (int k = 0; skipstage == mjhipSTAGE_NONE && k < m.nv; k++) {
    if (!(d.qLD[m.C_rowadr[k] + m.C_rownnz[k] - 1] >= mjh::MINVAL)) st |= MJHIP_INST_INERTIA;
  }
  if (st) status[inst] |= st;
}

// Batched mj_inverseSkip(POS / VEL) on the straight-line path: the generated k_va (POS) or
// k_acc (VEL) ran the remaining stages and, for an instance with constraint rows (made by the
// previous call), left the raw mj_rne(flg_acc = 1) in qfrc_inverse. Here those instances
// finish as the reference does on the rows it kept: mj_referenceConstraint when the velocity
// stage ran (POS), mj_invConstraint, then the assembly (engine_inverse.c:169-252).
// all != 0: a model whose rows serve every instance (contacts): the straight-line stage
// stored the raw RNE for every instance, which is assembled here, rows or none
// (mj_invConstraint with nefc = 0 zeroes qfrc_constraint, engine_inverse.c:168-177)
__global__ __launch_bounds__(64) void k_skip_rows(mjhipModel m, Mirror mr, int B, int skipstage,
                                                  double* __restrict__ qfrc_out, int all) {
  const long inst = (long)blockIdx.x*64 + threadIdx.x;
  if (inst >= B) return;
  Lane<64> d = lane_view(mr, blockIdx.x, threadIdx.x);
  if (!d.efc_count[0] && !all) return;
  if (d.efc_count[0] && skipstage == mjhipSTAGE_POS) mjh::referenceConstraint(m, d);
  mjh::invConstraint(m, d);
  for (int i = 0; i < m.nv; i++) {
    d.qfrc_inverse[i] += m.dof_armature[i] * d.qacc[i] - d.qfrc_passive[i] -
                         d.qfrc_constraint[i];
  }
  if (qfrc_out) {
    for (int i = 0; i < m.nv; i++) qfrc_out[inst*m.nv + i] = d.qfrc_inverse[i];
  }
}

// slider-crank/site/body transmissions, sensors and energy after the generated kernels and
// the constraint kernel (mjh::transmissionAfter, mjh::sensorsAfter)
__global__ __launch_bounds__(64) void k_sensors(mjhipModel m, Mirror mr, int B, int sensors,
                                                int trn) {
  const int blk = blockIdx.x, lane = threadIdx.x;
  if ((long)blk*64 + lane >= B) return;
  Lane<64> d = lane_view(mr, blk, lane);
  mjh::sensorsAfter<64>(m, d, sensors != 0, trn != 0);
}

// row-major (B x n) <-> mirror block layout
__global__ void k_to_mirror(const double* __restrict__ src, double* __restrict__ dst, int B,
                            int n) {
  long t = (long)blockIdx.x*blockDim.x + threadIdx.x;
  if (t >= (long)B*n) return;
  long inst = t / n, k = t % n;
  dst[((inst >> 6)*n + k)*64 + (inst & 63)] = src[t];
}

__global__ void k_from_mirror(const double* __restrict__ src, double* __restrict__ dst, int B,
                              int n) {
  long t = (long)blockIdx.x*blockDim.x + threadIdx.x;
  if (t >= (long)B*n) return;
  long inst = t / n, k = t % n;
  dst[t] = src[((inst >> 6)*n + k)*64 + (inst & 63)];
}

// mjd_inverseFD expansion (engine_derivative_fd.c:611-719): base state b and perturbation
// p (0 = centre, 1..nv = qacc_i + eps, nv+1..2nv = qvel_i + eps, 2nv+1..3nv = qpos
// integrated along e_i by eps). Instances are base-major: inst = b*(3nv+1) + p.
// Layout 1 (stage skipping, mj_inverseSkip(mjSTAGE_POS) for the qvel/qacc perturbations):
// the instances that run the position stage first -- the centres b, then the qpos
// perturbations nbase + b*nv + i (dof i) -- then from A = nbase*(nv+1) the others,
// A + b*2nv + (p-1). The centres lead so that they fill whole waves: only their mirror slots
// keep every field (Mirror::fd_elide, codegen.FD_KEEP).
// Layout 2 (the qacc perturbations run mj_inverseSkip(mjSTAGE_VEL), the qvel ones
// mjSTAGE_POS, engine_derivative_fd.c:646-699): the same position-stage block, then the qacc
// perturbations A + b*nv + (p-1), then the qvel ones A + nbase*nv + b*nv + (p-1-nv), so that
// each skip kernel covers whole waves of one kind.
__device__ static inline long fd_inst(int layout, long nbase, long b, int p, int nv) {
  if (!layout) return b*(3*nv + 1) + p;
  if (p == 0) return b;
  if (p > 2*nv) return nbase + b*nv + (p - 2*nv - 1);
  if (layout == 1) return nbase*(nv + 1) + b*2*nv + (p - 1);
  if (p <= nv) return nbase*(nv + 1) + b*nv + (p - 1);
  return nbase*(nv + 1) + nbase*nv + b*nv + (p - 1 - nv);
}

// instances [first, end) of the layout (first a multiple of 64), one block per 64 instances,
// its kExpandWaves waves taking turns over the input components: qvel[k], qacc[k] (k < nv), joint j's
// qpos (mj_integratePos on dof i for the qpos perturbations), ctrl[k]. The 64 lanes of a wave
// write one 512-byte mirror line per value. gate: the stage-skip fall-back's expansion (mjhip_inverseFDBatch): it runs only when
// k_vaskip found a centre with limit rows (fdflag[0]), and its first thread hands the range
// {first, end} -- or the empty {first, first} -- to the fall-back k_all (fdflag[1..2])
// the base state b and perturbation p of instance inst in the layout (the inverse of fd_inst)
__device__ static inline void fd_bp(int layout, long nbase, long inst, int nv, long* b, int* p) {
  const int P = 3*nv + 1;
  if (!layout) {
    *b = inst / P;
    *p = (int)(inst % P);
  } else if (inst < nbase) {
    *b = inst;
    *p = 0;
  } else if (inst < nbase*(nv + 1)) {
    const long t = inst - nbase;
    *b = t / nv;
    *p = 2*nv + 1 + (int)(t % nv);
  } else if (layout == 1) {
    const long t = inst - nbase*(nv + 1);
    *b = t / (2*nv);
    *p = 1 + (int)(t % (2*nv));
  } else {
    long t = inst - nbase*(nv + 1);
    const bool vel = t >= nbase*nv;
    if (vel) t -= nbase*nv;
    *b = t / nv;
    *p = 1 + (int)(t % nv) + (vel ? nv : 0);
  }
}

constexpr int kExpandWaves = 16;   // 4 measured 13 us per 28,672 instances (latency-bound)
__global__ __launch_bounds__(64*kExpandWaves) void k_fd_expand(mjhipModel m, Mirror mr, int nbase,
                                                  const double* __restrict__ qpos,
                                                  const double* __restrict__ qvel,
                                                  const double* __restrict__ qacc,
                                                  const double* __restrict__ ctrl, double eps,
                                                  int layout, int* __restrict__ fdflag,
                                                  long first, long end, int gate) {
  const int nv = m.nv, nq = m.nq, P = 3*nv + 1;
  const int ncomp = 2*nv + m.njnt + (ctrl ? m.nu : 0);
  // blocks of blockDim.x / 64 waves, striding over the 64-instance blocks of [first, end)
  // (the main expansion: one block each; the gated one: a few one-wave blocks, so that the
  // usual empty launch dispatches little): wave w writes components w, w + waves, ...
  const int lane = threadIdx.x % 64, wave = threadIdx.x / 64, waves = blockDim.x / 64;
  if (gate) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      fdflag[1] = (int)first;
      fdflag[2] = fdflag[0] ? (int)end : (int)first;
    }
    if (!fdflag[0]) return;
  } else if (fdflag && blockIdx.x == 0 && threadIdx.x == 0) {
    fdflag[0] = 0;                       // k_vaskip raises it later in stream order
    fdflag[3] = 0;                       // and k_fdall this one, should a wait time out
  }
  for (long blk = first/64 + blockIdx.x; blk*64 < end; blk += gridDim.x) {
  const long inst = blk*64 + lane;
  if (inst >= end || inst >= (long)nbase*P) continue;
  long b;
  int p;
  fd_bp(layout, nbase, inst, nv, &b, &p);
  Lane<64> d = lane_view(mr, (int)(inst >> 6), lane);
  for (int comp = wave; comp < ncomp; comp += waves) {
  if (comp < nv) {                       // qvel_k (+ eps on the qvel perturbation k)
    const double x = qvel[b*nv + comp];
    d.qvel[comp] = p - 1 - nv == comp ? x + eps : x;
    continue;
  }
  if (comp < 2*nv) {                     // qacc_k (+ eps on the qacc perturbation k)
    const int k = comp - nv;
    const double x = qacc[b*nv + k];
    d.qacc[k] = p - 1 == k ? x + eps : x;
    continue;
  }
  if (comp >= 2*nv + m.njnt) {           // flg_actuation: the base state's controls
    const int k = comp - 2*nv - m.njnt;
    d.ctrl[k] = ctrl[b*m.nu + k];
    continue;
  }
  // joint j's qpos: the base state's, or mj_integratePos(m, qpos, e_i, eps) for the qpos
  // perturbation of dof i (engine_support.c:1518-1550)
  const int j = comp - 2*nv, i = p > 2*nv ? p - 1 - 2*nv : -1;
  int padr = m.jnt_qposadr[j], vadr = m.jnt_dofadr[j], t = m.jnt_type[j];
  const long bq = b*nq;
  if (t == mjhipJNT_FREE) {
    for (int c = 0; c < 3; c++) {
      d.qpos[padr+c] = i < 0 ? qpos[bq + padr + c]
                             : qpos[bq + padr + c] + eps * (vadr + c == i ? 1.0 : 0.0);
    }
    padr += 3;
    vadr += 3;
    t = mjhipJNT_BALL;
  }
  if (t == mjhipJNT_BALL) {
    double q[4] = {qpos[bq + padr], qpos[bq + padr + 1], qpos[bq + padr + 2],
                   qpos[bq + padr + 3]};
    if (i >= 0) {
      const double vel[3] = {vadr == i ? 1.0 : 0.0, vadr + 1 == i ? 1.0 : 0.0,
                             vadr + 2 == i ? 1.0 : 0.0};
      mjh::quatIntegrate(q, vel, eps);
    }
    for (int c = 0; c < 4; c++) d.qpos[padr+c] = q[c];
  } else {
    d.qpos[padr] = i < 0 ? qpos[bq + padr] : qpos[bq + padr] + eps * (vadr == i ? 1.0 : 0.0);
  }
  }
  }
}

// diff(): DfD*[b][i][:] = (f(perturbed) - f(centre)) / eps  (engine_derivative_fd.c:48-53)
// Sensor rows follow the reference's stage skipping: a qacc perturbation runs
// mj_inverseSkip(mjSTAGE_VEL), so only acceleration-stage sensors change and the others keep
// the centre's values (their difference is exactly 0); a qvel perturbation runs
// mjSTAGE_POS, so position-stage sensors keep theirs (engine_derivative_fd.c:646-699).
// flg_actuation (inverseSkip, engine_derivative_fd.c:160-168): every evaluation's force is
// qfrc_inverse - qfrc_actuator, with mj_fwdActuation run after the inverse (k_fd_act)

__global__ void k_fd_act(mjhipModel m, Mirror mr, long ninst) {
  const long inst = (long)blockIdx.x*blockDim.x + threadIdx.x;
  if (inst >= ninst) return;
  Lane<64> d = lane_view(mr, (int)(inst >> 6), (int)(inst & 63));
  mjh::fwdActuation(m, d);
}

// DfDq/DfDv/DfDa (engine_derivative_fd.c:48-53) one thread per output element, the row's
// element k fastest, so a wave's stores are contiguous (the same difference and scaling as
// k_fd_diff, which keeps the sensor rows and DmDq; an LDS-tiled form, one block per 64
// instances, measured slower: 17.5 against 15.8 us at 1,024 base states)
__global__ void k_fd_dfd(mjhipModel m, Mirror mr, int nbase, double eps, int flg_actuation,
                         double* __restrict__ DfDq, double* __restrict__ DfDv,
                         double* __restrict__ DfDa, int layout) {
  const int nv = m.nv, P = 3*nv + 1;
  const long t = (long)blockIdx.x*blockDim.x + threadIdx.x;
  if (t >= (long)nbase*(P-1)*nv) return;
  const int k = (int)(t % nv);
  const long r = t / nv;
  const long b = r / (P-1);
  const int p = (int)(r % (P-1)) + 1;
  double* out;
  int i;
  if (p <= nv) {
    out = DfDa; i = p - 1;
  } else if (p <= 2*nv) {
    out = DfDv; i = p - 1 - nv;
  } else {
    out = DfDq; i = p - 1 - 2*nv;
  }
  if (!out) return;
  const long ic = fd_inst(layout, nbase, b, 0, nv), ip = fd_inst(layout, nbase, b, p, nv);
  Lane<64> c = lane_view(mr, (int)(ic >> 6), (int)(ic & 63));
  Lane<64> q = lane_view(mr, (int)(ip >> 6), (int)(ip & 63));
  double fq = q.qfrc_inverse[k], fc = c.qfrc_inverse[k];
  if (flg_actuation) {
    fq -= q.qfrc_actuator[k];
    fc -= c.qfrc_actuator[k];
  }
  out[(b*nv + i)*nv + k] = (1/eps) * (fq - fc);
}

__global__ void k_fd_diff(mjhipModel m, Mirror mr, int nbase, double eps, int flg_actuation,
                          double* __restrict__ DfDq, double* __restrict__ DfDv,
                          double* __restrict__ DfDa, double* __restrict__ DsDq,
                          double* __restrict__ DsDv, double* __restrict__ DsDa,
                          double* __restrict__ DmDq, int layout) {
  const int nv = m.nv, P = 3*nv + 1;
  long t = (long)blockIdx.x*blockDim.x + threadIdx.x;   // one thread per (b, perturbation)
  if (t >= (long)nbase*(P-1)) return;
  long b = t / (P-1);
  int p = (int)(t % (P-1)) + 1;
  long ic = fd_inst(layout, nbase, b, 0, nv), ip = fd_inst(layout, nbase, b, p, nv);
  Lane<64> c = lane_view(mr, (int)(ic >> 6), (int)(ic & 63));
  Lane<64> q = lane_view(mr, (int)(ip >> 6), (int)(ip & 63));
  double inv_h = 1/eps;
  double *out, *sout;
  int i, minstage;
  if (p <= nv) {
    out = DfDa; sout = DsDa; i = p - 1; minstage = mjhipSTAGE_ACC;
  } else if (p <= 2*nv) {
    out = DfDv; sout = DsDv; i = p - 1 - nv; minstage = mjhipSTAGE_VEL;
  } else {
    out = DfDq; sout = DsDq; i = p - 1 - 2*nv; minstage = mjhipSTAGE_POS;
  }
  if (out) {
    for (int k = 0; k < nv; k++) {
      double fq = q.qfrc_inverse[k], fc = c.qfrc_inverse[k];
      if (flg_actuation) {
        fq -= q.qfrc_actuator[k];
        fc -= c.qfrc_actuator[k];
      }
      out[(b*nv + i)*nv + k] = inv_h * (fq - fc);
    }
  }
  if (sout) {
    const int ns = m.nsensordata;
    for (int s = 0; s < m.nsensor; s++) {
      const bool ran = m.sensor_needstage[s] >= minstage;
      for (int k = m.sensor_adr[s]; k < m.sensor_adr[s] + m.sensor_dim[s]; k++) {
        const double x1 = c.sensordata[k], x2 = ran ? q.sensordata[k] : x1;
        sout[(b*nv + i)*ns + k] = inv_h * (x2 - x1);
      }
    }
  }
  if (DmDq && p > 2*nv) {
    for (int k = 0; k < m.nM; k++) {
      DmDq[(b*nv + i)*m.nM + k] = inv_h * (q.qM[k] - c.qM[k]);
    }
  }
}

// the mj_inverse assembly of a split launch (k_spos, then k_sfv beside k_constraint_coop on
// the second stream): qfrc_inverse = rne + ((armature*qacc - passive) - constraint), in the
// reference's order and with k_constraint_coop's own expression (engine_inverse.c:132-153),
// the constraint kernel's status bits, and the row-major output through LDS (coalesced)
// One thread per (instance, dof), block (blk, dof k) over the block's 64 instances: the mirror
// reads are whole 512-byte lines; the row-major writes of a block land in one 64 nv region.
__global__ __launch_bounds__(64) void k_assemble(mjhipModel m, Mirror mr, int B,
                                                 const int* __restrict__ cstat,
                                                 double* __restrict__ qfrc_out,
                                                 int* __restrict__ status) {
  const int nv = m.nv, blk = blockIdx.x / nv, k = blockIdx.x % nv, lane = threadIdx.x;
  const long inst = (long)blk*64 + lane;
  if (inst >= B) return;
  const long e = ((long)blk*nv + k)*64 + lane;       // the mirror's [blk][k][lane] element
  const double out = mr.qfrc_inverse[e] + (m.dof_armature[k] * mr.qacc[e] -
                                           mr.qfrc_passive[e] - mr.qfrc_constraint[e]);
  mr.qfrc_inverse[e] = out;
  if (qfrc_out) qfrc_out[inst*nv + k] = out;
  if (k == 0 && status && cstat[inst]) status[inst] |= cstat[inst];
}

// Constraint-free mj_forward over a batch (mjh::forwardSkip). Optional row-major qpos, qvel,
// ctrl are copied into the mirror first; qfrc_applied / xfrc_applied are read from the
// mirror; optional row-major qacc is written at the end.
template <bool CONTACT>
__global__ __launch_bounds__(64) void k_forward(mjhipModel m, Mirror mr, int B,
                                                const double* __restrict__ qpos_in,
                                                const double* __restrict__ qvel_in,
                                                const double* __restrict__ ctrl_in,
                                                double* __restrict__ qacc_out,
                                                int* __restrict__ status) {
  const int blk = blockIdx.x, lane = threadIdx.x;
  const long inst = (long)blk*64 + lane;
  if (inst >= B) return;
  Lane<64> d = lane_view(mr, blk, lane);
  if (qpos_in) {
    for (int k = 0; k < m.nq; k++) d.qpos[k] = qpos_in[inst*m.nq + k];
  }
  if (qvel_in) {
    for (int k = 0; k < m.nv; k++) d.qvel[k] = qvel_in[inst*m.nv + k];
  }
  if (ctrl_in) {
    for (int k = 0; k < m.nu; k++) d.ctrl[k] = ctrl_in[inst*m.nu + k];
  }
  int st = mjh::forwardSkip<64, CONTACT>(m, d, mjhipSTAGE_NONE);
  if (qacc_out) {
    for (int k = 0; k < m.nv; k++) qacc_out[inst*m.nv + k] = d.qacc[k];
  }
  if (status) status[inst] = st;
}

//==================================== host side ==============================================

static thread_local std::string g_last_error;
static void (*g_error_cb)(const char*) = nullptr;

static void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

#define HIPCHECK(expr)                                                              \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__,    \
                __LINE__);                                                          \
      return MJHIP_ERR_HIP;                                                         \
    }                                                                               \
  } while (0)

struct mjhipContext_ {
  int device = 0;
  int capacity = 0;         // instances (multiple of 64)
  int efc_cap = 0;
  int con_cap = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  mjhipModel hmodel{};      // host copy of sizes (pointers are host pointers of the caller)
  mjhipModel dmodel{};      // device pointers
  void* dmodel_buf = nullptr;
  Mirror mirror{};
  void* mirror_buf = nullptr;
  size_t mirror_bytes = 0;
  std::unordered_map<std::string, std::pair<double*, int>> fields;   // name -> (ptr, S)
  std::unordered_map<std::string, std::pair<int*, int>> ifields;   // int scratch fields
  std::unordered_set<std::string> contig;  // instance-contiguous fields (XSCC / XSIC)
  std::unordered_set<const void*> contig_ptr;   // and their device storage
  // staging for row-major host transfers
  double* stage = nullptr;
  size_t stage_bytes = 0;
  int* status = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  const FastKernelEntry* fast = nullptr;   // straight-line kernel for this model, if any
  int* worklist = nullptr;                 // capacity + 2 ints: [count0, count1, list...]
  int wl_parity = 0;                       // counter the next fast launch uses
  int wl_last = 0;                         // counter the last fast launch used
  int last_path = -1;                      // mjhip_contextLastPath
  const char* con_kernel = "none";         // mjhip_contextConstraintKernel
  // mjhip_inverseFDBatch's stage-skip fall-back, decided on the device: [0] a centre has limit
  // rows (k_vaskip), [1..2] the instance range {first, end} the gated k_fd_expand hands to
  // k_all
  int* fdflag = nullptr;
  int* fdflags = nullptr;                  // k_fdall's centre-block flags (capacity/64)
  int fd_epoch = 0;                        // the value k_fdall's flags are raised to
  CoopPair* pairs = nullptr;               // static geom-pair program (coop_program)
  mjh::ContactParam* cparams = nullptr;    // each program pair's mj_contactParam
  int* prog_ipair = nullptr;               // each program pair's predefined-pair index or -1
  unsigned long long* masks = nullptr;     // the cooperative kernel's chain masks (coop_masks)
  int npair = 0;
  bool boxpair = false;                    // a box-box pair is in the program (coop LDS)
  int coop = 16;                           // lanes per instance of k_constraint_coop (0: off)
  // the split launch (FastKernelEntry.launch_split): the cooperative constraint kernel on a
  // second stream beside the fac/va stages, joined by k_assemble; created on first use
  hipStream_t aux = nullptr;
  hipEvent_t evpos = nullptr, evcon = nullptr;
  int* cstat = nullptr;                    // the constraint kernel's status bits per instance
  bool spatial = false;                    // spatial tendons: k_tendon_after runs (post_pass.h)
  // a straight-line kernel specialized for this model at run time (mjhip_contextLoadKernel):
  // a gfx950 code object holding extern "C" k_all_<name>; rt.launch stays null
  unsigned long long sig = 0;              // model_signature of the model at creation
  hipModule_t rt_module = nullptr;
  hipFunction_t rt_fn = nullptr;
  FastKernelEntry rt{};
  std::string rt_name;
  hipDeviceptr_t rt_tbuf = nullptr;        // the code object's mjh_tbuf (null: none)
  // per-stage timers (mjhip_contextTimers): the device accumulator the phase marks add to,
  // the reference's mjTimerStat table, and the events around each timed call
  unsigned long long* tbuf = nullptr;
  mjhipTimerStat timer[mjhipNTIMER]{};
  unsigned long long traw[MJH_TSLOTS]{};   // the raw mark sums (tools/exp_phases.py)
  hipEvent_t tev0 = nullptr, tev1 = nullptr;
};

// FNV-1a 64 over sizes, options and every model array (= fields.model_signature in Python)
static unsigned long long model_signature(const mjhipModel* m) {
  unsigned long long h = 0xcbf29ce484222325ull;
  auto feed = [&](const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; i++) {
      h ^= b[i];
      h *= 0x100000001b3ull;
    }
  };
#define XS(name) { int v = m->name; feed(&v, 4); }
  MJHIP_MODEL_SIZES
#undef XS
  feed(&m->opt.timestep, 8);
  feed(&m->opt.impratio, 8);
  feed(m->opt.gravity, 24);
  feed(m->opt.wind, 24);
  feed(m->opt.magnetic, 24);
  feed(&m->opt.density, 8);
  feed(&m->opt.viscosity, 8);
  feed(&m->opt.o_margin, 8);
  feed(m->opt.o_solref, 16);
  feed(m->opt.o_solimp, 40);
  feed(m->opt.o_friction, 40);
  feed(&m->opt.integrator, 4);
  feed(&m->opt.cone, 4);
  feed(&m->opt.jacobian, 4);
  feed(&m->opt.disableflags, 4);
  feed(&m->opt.enableflags, 4);
  feed(&m->opt.ccd_tolerance, 8);
  feed(&m->opt.ccd_iterations, 4);
#define MJ_M(n) m->n
#define X(type, name, d0, d1) if (m->name) feed(m->name, sizeof(type) * (size_t)(m->d0) * (d1));
  MJHIP_MODEL_POINTERS
#undef X
#undef MJ_M
  return h;
}

// model features outside the device path: rejected at context creation (fail loudly)
static const char* unsupported(const mjhipModel* m) {
  if ((m->opt.enableflags & mjhipENBL_INVDISCRETE) && m->opt.integrator == mjhipINT_RK4) {
    return "mjENBL_INVDISCRETE with the RK4 integrator (an error in the reference)";
  }
  for (int i = 0; i < m->ntendon; i++) {
    for (int w = m->tendon_adr[i]; w < m->tendon_adr[i] + m->tendon_num[i]; w++) {
      if (m->wrap_type[w] < mjhipWRAP_JOINT || m->wrap_type[w] > mjhipWRAP_CYLINDER) {
        return "unknown tendon wrap object type";
      }
    }
  }
  for (int i = 0; i < m->nu; i++) {
    int t = m->actuator_trntype[i];
    if (t != mjhipTRN_JOINT && t != mjhipTRN_JOINTINPARENT && t != mjhipTRN_TENDON &&
        t != mjhipTRN_SLIDERCRANK && t != mjhipTRN_SITE && t != mjhipTRN_BODY) {
      return "unknown transmission type";
    }
  }
  if (mjh_isSparse(m)) {
    for (int i = 0; i < m->nu; i++) {
      if (m->actuator_trntype[i] == mjhipTRN_TENDON &&
          m->wrap_type[m->tendon_adr[m->actuator_trnid[2*i]]] != mjhipWRAP_JOINT) {
        // the reference's moment row is the tendon's compressed ten_J row (:1060-1067), whose
        // pattern follows the wrapping state; actuator_moment's pattern is model-constant here
        return "a spatial-tendon transmission in a sparse-Jacobian model";
      }
    }
  }
  for (int i = 0; i < m->nsensor; i++) {
    const int t = m->sensor_type[i];
    if (t > mjhSENS_CLOCK) return "plugin/user sensors";
    if (t >= mjhSENS_GEOMDIST && t <= mjhSENS_GEOMFROMTO) {
      // mj_geomDistance's functions outside the subset: meshes, height fields, SDFs, and
      // libccd's MPR (convex and box-box pairs with the native solver disabled)
      const int o = m->sensor_objid[i], r = m->sensor_refid[i];
      const int n1 = m->sensor_objtype[i] == 1 ? m->body_geomnum[o] : 1;
      const int a1 = m->sensor_objtype[i] == 1 ? m->body_geomadr[o] : o;
      const int n2 = m->sensor_reftype[i] == 1 ? m->body_geomnum[r] : 1;
      const int a2 = m->sensor_reftype[i] == 1 ? m->body_geomadr[r] : r;
      const bool nccd = !(m->opt.disableflags & mjhipDSBL_NATIVECCD);
      for (int g1 = a1; g1 < a1 + n1; g1++) {
        for (int g2 = a2; g2 < a2 + n2; g2++) {
          int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
          if (t1 > t2) std::swap(t1, t2);
          const bool ccd = mjhip_isConvexPair(t1, t2) ||
                           (t1 == mjhipGEOM_BOX && t2 == mjhipGEOM_BOX);
          if ((ccd && !nccd) || (!ccd && mjhip_pairMaxContacts(m, t1, t2) < 0)) {
            return "a geom-distance sensor on a height field or SDF geom, or on a "
                   "convex pair with the native CCD solver disabled";
          }
        }
      }
    }
    if (t == mjhSENS_RANGEFINDER) {   // mj_ray's SDF path is not built
      const int body = m->site_bodyid[m->sensor_objid[i]];
      for (int g = 0; g < m->ngeom; g++) {
        if (m->geom_type[g] == mjhipGEOM_SDF && !mjh::rayEliminate(*m, g, body)) {
          return "a rangefinder that can see an SDF geom";
        }
      }
    }
  }
  return nullptr;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" {

MJHIP_API const char* mjhip_version(void) { return "mjhip 0.1 (gfx950)"; }

#ifdef MJH_PHASE_TIMING
// experiment builds only (tools/exp_phases.py): the raw phase-mark sums of a timed context
extern "C" int mjhip_phaseRead(mjhipContext* c, unsigned long long* out) {
  if (!c) return 1;
  memcpy(out, c->traw, sizeof(c->traw));
  memset(c->traw, 0, sizeof(c->traw));
  return 0;
}
#endif

MJHIP_API const char* mjhip_lastError(void) { return g_last_error.c_str(); }

MJHIP_API void mjhip_setErrorCallback(void (*cb)(const char* msg)) { g_error_cb = cb; }

MJHIP_API int mjhip_deviceCount(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

MJHIP_API int mjhip_fieldSize(const mjhipModel* m, const char* name) {
#define MJ_M(n) m->n
#define XD(nm, d0, d1, stage) if (!strcmp(name, #nm)) return (m->d0) * (d1);
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
#undef XD
#undef MJ_M
  return -1;
}

MJHIP_API int mjhip_outputDoubles(const mjhipModel* m) {
  int w = 0;
#define MJ_M(n) m->n
#define XD(nm, d0, d1, stage) if (stage > 0) w += (m->d0) * (d1);
  MJHIP_DATA_FIELDS
#undef XD
#undef MJ_M
  return w;
}

MJHIP_API int mjhip_contextCreate(const mjhipModel* m, int device, int capacity,
                                  mjhipContext** out) {
  return mjhip_contextCreateCapped(m, device, capacity, 0, 0, out);
}

MJHIP_API int mjhip_contextCreateCapped(const mjhipModel* m, int device, int capacity,
                                        int max_contacts, int max_rows, mjhipContext** out) {
  if (!m || !out || capacity <= 0 || max_contacts < 0 || max_rows < 0) {
    set_error("mjhip_contextCreate: bad argument");
    return MJHIP_ERR_ARG;
  }
  *out = nullptr;
  int ndev = mjhip_deviceCount();
  if (ndev <= 0) {
    set_error("no HIP device available (the engine has no CPU fallback)");
    return MJHIP_ERR_NO_DEVICE;
  }
  if (device < 0 || device >= ndev) {
    set_error("device %d out of range (%d devices)", device, ndev);
    return MJHIP_ERR_ARG;
  }
  if (const char* why = unsupported(m)) {
    set_error("model uses a feature the device path does not support: %s", why);
    return MJHIP_ERR_MODEL;
  }
  HIPCHECK(hipSetDevice(device));
  mjhipContext* c = new mjhipContext_();
  c->device = device;
  c->capacity = (capacity + 63) & ~63;
  c->efc_cap = mjhip_efcCapacity(m);
  c->con_cap = mjhip_contactCapacity(m, nullptr);
  // caller caps (the reference's <size nconmax njmax> / arena bound): an instance that needs
  // more is flagged MJHIP_INST_CNSTRFULL, as mjWARN_CONTACTFULL / mjWARN_CNSTRFULL
  if (max_contacts && max_contacts < c->con_cap) c->con_cap = max_contacts;
  if (max_rows && max_rows < c->efc_cap) c->efc_cap = max_rows;
  c->hmodel = *m;

  // ---- model upload: one buffer, 256-byte aligned arrays
  size_t total = 0;
#define MJ_M(n) m->n
#define X(type, name, d0, d1) total += align256(sizeof(type) * (size_t)(m->d0) * (d1));
  MJHIP_MODEL_POINTERS
#undef X
  std::vector<char> hbuf(total > 0 ? total : 1, 0);
  size_t off = 0;
  c->dmodel = *m;
  if (hipMalloc(&c->dmodel_buf, hbuf.size()) != hipSuccess) {
    set_error("hipMalloc(model) failed");
    delete c;
    return MJHIP_ERR_HIP;
  }
#define X(type, name, d0, d1)                                                       \
  {                                                                                 \
    size_t nb = sizeof(type) * (size_t)(m->d0) * (d1);                              \
    if (nb && m->name) memcpy(hbuf.data() + off, m->name, nb);                      \
    c->dmodel.name = (type*)((char*)c->dmodel_buf + off);                           \
    off += align256(nb);                                                            \
  }
  MJHIP_MODEL_POINTERS
#undef X
#undef MJ_M
  if (hipMemcpy(c->dmodel_buf, hbuf.data(), hbuf.size(), hipMemcpyHostToDevice) != hipSuccess) {
    set_error("model upload failed");
    hipFree(c->dmodel_buf);
    delete c;
    return MJHIP_ERR_HIP;
  }

  // ---- mirror: per-instance fields in 64-instance blocks
  const size_t nblk = c->capacity / 64;
  size_t mb = 0;
  const int nv = m->nv, nbody = m->nbody, efc_cap = c->efc_cap, con_cap = c->con_cap;
  (void)nbody;
#define MJ_M(n) m->n
#define XD(name, d0, d1, stage) c->mirror.name##_n = (m->d0) * (d1); \
  mb += align256(sizeof(double) * nblk * 64 * (size_t)c->mirror.name##_n);
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
#undef XD
#define XSC(name, n) { const int nbody = m->nbody; (void)nbody; c->mirror.name##_n = (n); \
  mb += align256(sizeof(double) * nblk * 64 * (size_t)c->mirror.name##_n); }
  MJHIP_SCRATCH_FIELDS
#undef XSC
#define XSI(name, n) { c->mirror.name##_n = (n); \
  mb += align256(sizeof(int) * nblk * 64 * (size_t)c->mirror.name##_n); }
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
  (void)nv; (void)efc_cap; (void)con_cap;
  c->mirror.efc_cap = c->efc_cap;
  c->mirror.con_cap = c->con_cap;
  c->mirror.nj_cap = mjh_njCap(m, c->efc_cap);
  c->mirror_bytes = mb;
  if (hipMalloc(&c->mirror_buf, mb) != hipSuccess) {
    set_error("hipMalloc(mirror, %zu bytes) failed", mb);
    hipFree(c->dmodel_buf);
    delete c;
    return MJHIP_ERR_HIP;
  }
  hipMemset(c->mirror_buf, 0, mb);
  char* p = (char*)c->mirror_buf;
#define XD(name, d0, d1, stage) c->mirror.name = (double*)p; \
  c->fields[#name] = {c->mirror.name, c->mirror.name##_n}; \
  p += align256(sizeof(double) * nblk * 64 * (size_t)c->mirror.name##_n);
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
#undef XD
#define XSC(name, n) c->mirror.name = (double*)p; \
  c->fields[#name] = {c->mirror.name, c->mirror.name##_n}; \
  p += align256(sizeof(double) * nblk * 64 * (size_t)c->mirror.name##_n);
#undef XSCC
#define XSCC(name, n) c->contig.insert(#name); \
  if (c->mirror.name##_n > 0) c->contig_ptr.insert(p); XSC(name, n)
  MJHIP_SCRATCH_FIELDS
#undef XSC
#define XSI(name, n) c->mirror.name = (int*)p; \
  c->ifields[#name] = {c->mirror.name, c->mirror.name##_n}; \
  p += align256(sizeof(int) * nblk * 64 * (size_t)c->mirror.name##_n);
#undef XSIC
#define XSIC(name, n) c->contig.insert(#name); \
  if (c->mirror.name##_n > 0) c->contig_ptr.insert(p); XSI(name, n)
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
#undef XSCC
#undef XSIC
#define XSCC(name, n) XSC(name, n)
#define XSIC(name, n) XSI(name, n)
#undef MJ_M
  // every failure below releases the partial context through mjhip_contextFree
  auto fail = [&](const char* what) {
    set_error("%s failed", what);
    mjhip_contextFree(c);
    return MJHIP_ERR_HIP;
  };
  // staging: row-major qpos, qvel, qacc, qfrc for `capacity` instances
  c->stage_bytes = sizeof(double) * (size_t)c->capacity * (m->nq + 3*(size_t)m->nv + m->nu);
  if (hipMalloc((void**)&c->stage, c->stage_bytes) != hipSuccess ||
      hipMalloc((void**)&c->status, sizeof(int) * (size_t)c->capacity) != hipSuccess) {
    return fail("hipMalloc(staging)");
  }
  if (hipMalloc((void**)&c->worklist, sizeof(int) * ((size_t)c->capacity + 2)) != hipSuccess ||
      hipMemset(c->worklist, 0, 2 * sizeof(int)) != hipSuccess) {
    return fail("hipMalloc(worklist)");
  }
  if (hipMalloc((void**)&c->fdflag, 4 * sizeof(int)) != hipSuccess ||
      hipMemset(c->fdflag, 0, 4 * sizeof(int)) != hipSuccess) {
    return fail("hipMalloc(FD flag)");
  }
  const char* nofast = getenv("MJHIP_DISABLE_FAST");
  c->sig = model_signature(m);
  if (!(nofast && nofast[0] == '1')) {
    for (const FastKernelEntry* e = mjhip_fastKernels(); e->launch; e++) {
      if (e->sig == c->sig) c->fast = e;
    }
  }
  // the cooperative constraint kernel's pair program (16 lanes per instance: 8 and 32 were
  // slower, profiles/r02/bench_c4_L*.json; MJHIP_COOP_LANES=0 selects the one-lane
  // k_constraint)
  if (const char* lanes = getenv("MJHIP_COOP_LANES")) {
    const int n = atoi(lanes);             // 8 and 32: the contact path's lane-count variants
    c->coop = n == 0 ? 0 : (n == 8 || n == 32) ? n : 16;
  }
  if (c->con_cap > 0) {
    // the static collision program (csrc/pair_program.h): the cooperative kernel's pair
    // program, and collision()'s candidate list in every other kernel (Mirror::prog)
    std::vector<ProgItem> pairs = collision_pairs(m);
    c->npair = (int)pairs.size();
    for (const ProgItem& pr : pairs) {
      c->boxpair |= m->geom_type[pr.g1] == mjhipGEOM_BOX && m->geom_type[pr.g2] == mjhipGEOM_BOX;
    }
    if (c->npair) {
      const std::vector<CoopPair> prog = coop_program(m, pairs);
      // contact parameters are model constants: formed here once per pair, by the same
      // function (host arithmetic, as the reference's)
      const std::vector<mjh::ContactParam> cps = program_params(m, prog, pairs);
      std::vector<int> ipair(pairs.size());
      for (size_t i = 0; i < pairs.size(); i++) ipair[i] = pairs[i].ipair;
      if (hipMalloc((void**)&c->pairs, sizeof(CoopPair) * prog.size()) != hipSuccess ||
          hipMemcpy(c->pairs, prog.data(), sizeof(CoopPair) * prog.size(),
                    hipMemcpyHostToDevice) != hipSuccess ||
          hipMalloc((void**)&c->cparams, sizeof(mjh::ContactParam) * cps.size()) != hipSuccess ||
          hipMemcpy(c->cparams, cps.data(), sizeof(mjh::ContactParam) * cps.size(),
                    hipMemcpyHostToDevice) != hipSuccess ||
          hipMalloc((void**)&c->prog_ipair, sizeof(int) * ipair.size()) != hipSuccess ||
          hipMemcpy(c->prog_ipair, ipair.data(), sizeof(int) * ipair.size(),
                    hipMemcpyHostToDevice) != hipSuccess) {
        return fail("pair program upload");
      }
    }
  }
  c->mirror.prog = c->npair ? c->pairs : nullptr;
  c->mirror.prog_ipair = c->npair ? c->prog_ipair : nullptr;
  c->mirror.nprog = c->npair;
  // the native convex solver keeps its polytope in the instance's scratch: one lane per
  // instance (the cooperative kernel would run several pairs of an instance at once)
  if (mjh_needConvex(m) || m->nmesh || m->nhfield) c->coop = 0;
  c->spatial = mjh::hasSpatial(*m);
  // the cooperative kernel's per-dof chain masks are 64-bit
  if (m->nv > 64) c->coop = 0;
  if (c->coop) {
    // chain masks (mjh::chainMask per body: the body and its ancestors), then per body the
    // dofs of those bodies: model constants, formed here once
    std::vector<unsigned long long> mk(2 * (size_t)m->nbody, 0);
    for (int b = 0; b < m->nbody && b < 64; b++) mk[b] = mjh::chainMask(*m, b);
    for (int b = 0; b < m->nbody && b < 64; b++) {
      for (int j = 0; j < m->nv; j++) {
        if ((mk[b] >> m->dof_bodyid[j]) & 1) mk[m->nbody + b] |= 1ull << j;
      }
    }
    if (hipMalloc((void**)&c->masks, sizeof(unsigned long long) * mk.size()) != hipSuccess ||
        hipMemcpy(c->masks, mk.data(), sizeof(unsigned long long) * mk.size(),
                  hipMemcpyHostToDevice) != hipSuccess) {
      return fail("chain mask upload");
    }
  }
  if (c->coop) {
    // the cooperative kernel's dynamic LDS must fit one block: many box pairs (a large
    // efc_cap) or few lanes per instance can exceed it, and then the one-lane k_constraint
    // serves the model instead of every launch failing
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fail("hipGetDeviceProperties");
    if (coopLdsBytes(*m, c->coop, c->efc_cap, c->boxpair, c->npair, c->con_cap) >
        (unsigned)prop.sharedMemPerBlock) {
      c->coop = 0;
    }
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    return fail("hipStreamCreate");
  }
  c->own_stream = true;
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    return fail("hipEventCreate");
  }
  *out = c;
  return MJHIP_OK;
}

static int timers_detach(mjhipContext* c);
// the one context per process whose accumulator the phase marks may add into: mjh_tbuf is a
// process-wide device global per unit, so a second context's kernels would add into the
// first's accumulator
static mjhipContext* g_timed_ctx = nullptr;

MJHIP_API void mjhip_contextFree(mjhipContext* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  // the timer pointers go back to null while the stream still exists (timers_attach
  // synchronizes it); an accumulator some unit may still point at is leaked, not freed
  const bool detached = !c->tbuf || timers_detach(c) == MJHIP_OK;
  if (g_timed_ctx == c) g_timed_ctx = nullptr;
  if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
  if (c->aux) {
    hipStreamSynchronize(c->aux);
    hipStreamDestroy(c->aux);
  }
  if (c->evpos) hipEventDestroy(c->evpos);
  if (c->evcon) hipEventDestroy(c->evcon);
  hipFree(c->cstat);
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  if (c->tev0) hipEventDestroy(c->tev0);
  if (c->tev1) hipEventDestroy(c->tev1);
  if (detached) hipFree(c->tbuf);
  hipFree(c->stage);
  hipFree(c->status);
  hipFree(c->worklist);
  hipFree(c->fdflag);
  hipFree(c->fdflags);
  hipFree(c->pairs);
  hipFree(c->cparams);
  hipFree(c->prog_ipair);
  hipFree(c->masks);
  hipFree(c->mirror_buf);
  hipFree(c->dmodel_buf);
  if (c->rt_module) hipModuleUnload(c->rt_module);
  delete c;
}

MJHIP_API int mjhip_contextLoadKernel(mjhipContext* c, const void* image, size_t size,
                                      const char* name, unsigned long long signature,
                                      int cmode) {
  if (!c || !image || !size || !name || cmode < 0 || cmode > 2) {
    set_error("mjhip_contextLoadKernel: bad arguments");
    return MJHIP_ERR_ARG;
  }
  if (signature != c->sig) {
    set_error("mjhip_contextLoadKernel: kernel '%s' was generated for another model "
              "(signature %016llx, context %016llx)", name, signature, c->sig);
    return MJHIP_ERR_MODEL;
  }
  if (mjh_isSparse(&c->hmodel)) {
    // the straight-line kernels and their constraint kernels keep dense rows
    set_error("mjhip_contextLoadKernel: sparse-Jacobian models run the generic kernel");
    return MJHIP_ERR_MODEL;
  }
  hipSetDevice(c->device);
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  const std::string kname = std::string("k_all_") + name;
  if (hipModuleLoadData(&mod, image) != hipSuccess) {
    set_error("mjhip_contextLoadKernel: hipModuleLoadData failed (not a gfx950 code object?)");
    return MJHIP_ERR_HIP;
  }
  if (hipModuleGetFunction(&fn, mod, kname.c_str()) != hipSuccess) {
    hipModuleUnload(mod);
    set_error("mjhip_contextLoadKernel: no kernel '%s' in the code object", kname.c_str());
    return MJHIP_ERR_HIP;
  }
  if (c->rt_module) hipModuleUnload(c->rt_module);
  c->rt_module = mod;
  c->rt_fn = fn;
  size_t tbytes = 0;                       // its per-stage timer pointer (MJH_TBUF_EXTERN)
  if (hipModuleGetGlobal(&c->rt_tbuf, &tbytes, mod, "mjh_tbuf") != hipSuccess ||
      tbytes != sizeof(void*)) {
    c->rt_tbuf = nullptr;
    (void)hipGetLastError();
  }
  c->rt_name = name;
  c->rt = FastKernelEntry{signature, nullptr, c->rt_name.c_str(), cmode};
  c->fast = &c->rt;
  c->wl_parity = 0;                        // the run-time kernel zeroes the counters as the
  return hipMemset(c->worklist, 0, 2 * sizeof(int)) == hipSuccess ? MJHIP_OK : MJHIP_ERR_HIP;
}

MJHIP_API int mjhip_ccdBatch(mjhipContext* c, int n, const int* g1, const int* g2,
                             const mjtNum* pos1, const mjtNum* mat1, const mjtNum* pos2,
                             const mjtNum* mat2, const mjtNum* margin, int max_iterations,
                             mjtNum tolerance, int max_contacts, mjtNum dist_cutoff,
                             mjtNum* dist, int* nx, mjtNum* x1, mjtNum* x2) {
  if (!c || n < 0 || (n && (!g1 || !g2 || !pos1 || !mat1 || !pos2 || !mat2 || !dist || !nx ||
                            !x1 || !x2)) || max_iterations < 1 || max_contacts < 0) {
    set_error("mjhip_ccdBatch: bad argument");
    return MJHIP_ERR_ARG;
  }
  // witness points kept per pair: mjCCDStatus holds mjMAXCONPAIR
  const int xcap = max_contacts <= 1 ? 1 :
                   (max_contacts < mjh::CCD_MAXCON ? max_contacts : mjh::CCD_MAXCON);
  if (!n) return MJHIP_OK;
  const int ng = c->hmodel.ngeom;
  for (int i = 0; i < n; i++) {            // every index the kernel reads, checked here
    if (g1[i] < 0 || g1[i] >= ng || g2[i] < 0 || g2[i] >= ng) {
      set_error("mjhip_ccdBatch: geom id out of range at pair %d", i);
      return MJHIP_ERR_ARG;
    }
  }
  HIPCHECK(hipSetDevice(c->device));
  const long nd = mjh::ccdScratchDoubles(max_iterations), ni = mjh::ccdScratchInts(max_iterations);
  std::vector<double> in(24L*n), out(kCcdOut*n);
  for (int i = 0; i < n; i++) {
    memcpy(&in[24L*i], pos1 + 3L*i, 3*sizeof(double));
    memcpy(&in[24L*i + 3], mat1 + 9L*i, 9*sizeof(double));
    memcpy(&in[24L*i + 12], pos2 + 3L*i, 3*sizeof(double));
    memcpy(&in[24L*i + 15], mat2 + 9L*i, 9*sizeof(double));
  }
  // one allocation: inputs, margins, outputs, scratch, then the int arrays
  const size_t bytes = sizeof(double)*(24L*n + n + kCcdOut*n + nd*n) +
                       sizeof(int)*(2L*n + ni*n + n);
  char* buf = nullptr;
  HIPCHECK(hipMalloc((void**)&buf, bytes));
  double* d_in = (double*)buf;
  double* d_margin = d_in + 24L*n;
  double* d_out = d_margin + n;
  double* d_x = d_out + kCcdOut*n;
  int* d_g = (int*)(d_x + nd*n);
  int* d_xi = d_g + 2L*n;
  int* d_bad = d_xi + ni*n;
  std::vector<double> mg(n, 0.0);
  if (margin) memcpy(mg.data(), margin, n*sizeof(double));
  std::vector<int> bad(n);
  int rc = MJHIP_OK;
  auto run = [&]() -> int {
    HIPCHECK(hipMemcpy(d_in, in.data(), 24L*n*sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_margin, mg.data(), n*sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_g, g1, n*sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_g + n, g2, n*sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemset(d_bad, 0, n*sizeof(int)));
    if (mjhip_launchCcd(c->stream, c->dmodel, n, d_g, d_g + n, d_in, d_margin, max_iterations,
                        tolerance, max_contacts, dist_cutoff, d_x, d_xi, d_out, d_bad)) {
      set_error("mjhip_ccdBatch: kernel launch failed");
      return MJHIP_ERR_HIP;
    }
    HIPCHECK(hipStreamSynchronize(c->stream));
    HIPCHECK(hipMemcpy(out.data(), d_out, kCcdOut*n*sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(bad.data(), d_bad, n*sizeof(int), hipMemcpyDeviceToHost));
    return MJHIP_OK;
  };
  rc = run();
  hipFree(buf);
  if (rc) return rc;
  for (int i = 0; i < n; i++) {
    if (bad[i]) {
      set_error(bad[i] == 1 ? "mjhip_ccdBatch: pair %d outgrew the solver's polytope capacity"
                            : "mjhip_ccdBatch: pair %d needs multicontact outside the built "
                              "subset (a shape other than a box or mesh, or a mesh polygon "
                              "or vertex fan over 16)", i);
      return MJHIP_ERR_MODEL;
    }
    const double* o = &out[kCcdOut*i];
    dist[i] = o[0];
    nx[i] = (int)o[1];
    const int k = nx[i] < xcap ? (nx[i] > 1 ? nx[i] : 1) : xcap;
    memcpy(x1 + 3L*xcap*i, o + 2, 3*k*sizeof(double));
    memcpy(x2 + 3L*xcap*i, o + 2 + 3*mjh::CCD_MAXCON, 3*k*sizeof(double));
  }
  return MJHIP_OK;
}

MJHIP_API int mjhip_contextCapacity(const mjhipContext* c) { return c ? c->capacity : 0; }

MJHIP_API const char* mjhip_contextFastKernel(const mjhipContext* c) {
  return (c && c->fast) ? c->fast->name : nullptr;
}

MJHIP_API int mjhip_contextLastPath(const mjhipContext* c) { return c ? c->last_path : -1; }

MJHIP_API const char* mjhip_contextConstraintKernel(const mjhipContext* c) {
  return c ? c->con_kernel : nullptr;
}

MJHIP_API int mjhip_worklistCount(mjhipContext* c) {
  if (!c) return -1;
  int n = 0;
  if (hipMemcpy(&n, c->worklist + c->wl_last, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}

MJHIP_API void* mjhip_contextStream(mjhipContext* c) { return c ? (void*)c->stream : nullptr; }

MJHIP_API int mjhip_contextSetStream(mjhipContext* c, void* stream) {
  if (!c) return MJHIP_ERR_ARG;
  if (c->own_stream && c->stream) {
    hipStreamSynchronize(c->stream);
    hipStreamDestroy(c->stream);
  }
  c->stream = (hipStream_t)stream;
  c->own_stream = false;
  return MJHIP_OK;
}

// the split launch of a contact model is opt-in (MJHIP_SPLIT=1): measured slower than the
// one-stream path at config 4, kept for the experiment
static bool split_disabled() {
  const char* e = getenv("MJHIP_SPLIT");
  return !(e && e[0] == '1');
}

// the split launch's second stream, its two events and the status-bit buffer (first use)
static int split_ready(mjhipContext* c) {
  if (c->aux) return MJHIP_OK;
  HIPCHECK(hipMalloc((void**)&c->cstat, sizeof(int)*(size_t)c->capacity));
  HIPCHECK(hipEventCreateWithFlags(&c->evpos, hipEventDisableTiming));
  HIPCHECK(hipEventCreateWithFlags(&c->evcon, hipEventDisableTiming));
  HIPCHECK(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
  return MJHIP_OK;
}

// the straight-line path's passes after the constraint part: sensors (and the transmission
// and energy terms they carry), INVDISCRETE's qacc restore, the status checks; then the
// work-list counters change hands
static int finish_fast(mjhipContext* c, int B, dim3 grid, dim3 block, int skipsensor,
                       int* status, bool discrete) {
  const int sensors = !skipsensor && c->hmodel.nsensor > 0 &&
                      !(c->hmodel.opt.disableflags & mjhipDSBL_SENSOR);
  const int trn = mjh_needTrnAfter(&c->hmodel) && !discrete;   // discrete: already formed
  if (sensors || trn || (c->hmodel.opt.enableflags & mjhipENBL_ENERGY)) {
    hipLaunchKernelGGL(k_sensors, grid, block, 0, c->stream, c->dmodel, c->mirror, B,
                       sensors, trn);
    HIPCHECK(hipGetLastError());
  }
  if (discrete) {                        // the caller's qacc back, after mj_sensorAcc
    hipLaunchKernelGGL(k_discrete_restore, grid, block, 0, c->stream, c->dmodel, c->mirror, B);
  }
  if (status) {
    hipLaunchKernelGGL(k_check, grid, block, 0, c->stream, c->dmodel, c->mirror, B, status,
                       (int)mjhipSTAGE_NONE);
    HIPCHECK(hipGetLastError());
  }
  c->wl_last = c->wl_parity;
  c->wl_parity ^= 1;
  return MJHIP_OK;
}

// internal launch_inverse flag (not a public MJHIP_FLAG_*): run the straight-line kernel of a
// work-list model without its constraint kernel; the next launch_inverse call continues the
// same work-list and serves both (the bare pipeline only: the FD stage-skip layout)
constexpr int kFlagDeferRows = 1 << 30;
// internal mjhip_inverseFDBatchEx flag: no stage-skip layout (every instance base-major, every
// field stored): the single-instance mjd_inverseFD reads back its last evaluation's fields
constexpr int kFlagFDFull = 1 << 29;

// range: null, or a device-side instance range {first, end} for the straight-line kernel (B
// then only sizes the grid: end - first <= B); only the FD fall-back uses it, on models whose
// whole pipeline is the straight-line and constraint kernels
static int launch_inverse(mjhipContext* c, int B, const double* qpos, const double* qvel,
                          const double* qacc, double* qfrc, int skipstage, int* status,
                          int flags = 0, int skipsensor = 0, const int* range = nullptr) {
  dim3 grid((B + 63) / 64), block(64);
  if (range && (skipstage != mjhipSTAGE_NONE || !c->fast || (flags & MJHIP_FLAG_GENERIC) ||
                status || qpos || qfrc || c->spatial || mjh::hasFluid(c->hmodel) ||
                mjh::hasDiscrete(c->hmodel) || mjh_needTrnAfter(&c->hmodel) || !skipsensor ||
                (c->hmodel.opt.enableflags & mjhipENBL_ENERGY))) {
    set_error("launch_inverse: a device-side range needs the bare straight-line pipeline");
    return MJHIP_ERR_ARG;
  }
  c->last_path = 0;
  if (skipstage == mjhipSTAGE_NONE && c->fast && !(flags & MJHIP_FLAG_GENERIC)) {
    c->last_path = 1;
    // two work-list counters alternate: this launch counts into `cnt` (zeroed by the
    // previous launch's k_pos, or at context creation) and zeroes `nxt` for the next one
    int* cnt = c->worklist + c->wl_parity;
    int* nxt = c->worklist + (c->wl_parity ^ 1);
    const bool discrete = mjh::hasDiscrete(c->hmodel);
    // fused rows whenever nbody allows, INVDISCRETE included (post_pass.h fastFusedOk)
    const bool fused = mjh::fastFusedOk(c->dmodel);
    if (c->fast->launch_split && !range && fused && c->coop && c->fast->cmode == 2 &&
        c->con_cap > 0 && !c->spatial && !mjh::hasFluid(c->dmodel) && !discrete &&
        !split_disabled()) {
      // rows on every instance: the position stage, then the cooperative constraint kernel
      // (position-stage outputs and inputs only) on the second stream beside the fac / va
      // stages, joined by the assembly
      if (const int rc = split_ready(c)) return rc;
      c->last_path = 3;
      const int* wl = c->worklist + 2;
      c->fast->launch_split(c->stream, c->mirror, B, 0, qpos, qvel, qacc, status, nxt,
                            c->mirror.efc_count);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipEventRecord(c->evpos, c->stream));
      // the fac / va stages are queued first: their 64-lane waves need a whole SIMD's
      // registers, which the constraint kernel's waves would otherwise take
      c->fast->launch_split(c->stream, c->mirror, B, 1, nullptr, nullptr, nullptr, status, nxt,
                            c->mirror.efc_count);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipStreamWaitEvent(c->aux, c->evpos, 0));
#define MJHIP_LAUNCH_COOP_SPLIT(G, X)                                                         \
      hipLaunchKernelGGL((k_constraint_coop<G, true, false, X>), dim3(coopGrid(B, G, false)),   \
                         dim3(64), coopLdsBytes(c->dmodel, G, c->efc_cap, c->boxpair,         \
                                                      c->npair, c->con_cap),                  \
                         c->aux, c->dmodel, c->mirror, B, wl, (const int*)cnt, c->pairs,      \
                         c->cparams, c->masks, c->npair, nullptr, nullptr, c->cstat)
      if (c->boxpair) MJHIP_LAUNCH_COOP_SPLIT(16, true);
      else if (c->coop == 8) MJHIP_LAUNCH_COOP_SPLIT(8, false);
      else if (c->coop == 32) MJHIP_LAUNCH_COOP_SPLIT(32, false);
      else MJHIP_LAUNCH_COOP_SPLIT(16, false);
#undef MJHIP_LAUNCH_COOP_SPLIT
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipEventRecord(c->evcon, c->aux));
      HIPCHECK(hipStreamWaitEvent(c->stream, c->evcon, 0));
      hipLaunchKernelGGL(k_assemble, dim3(grid.x*c->hmodel.nv), block, 0, c->stream, c->dmodel,
                         c->mirror, B, c->cstat, qfrc, status);
      HIPCHECK(hipGetLastError());
      return finish_fast(c, B, grid, block, skipsensor, status, false);
    }
    if (c->fast->launch) {
      c->fast->launch(grid, block, c->stream, c->mirror, B, qpos, qvel, qacc, qfrc, status,
                      c->worklist + 2, cnt, nxt, c->mirror.efc_count, range);
      HIPCHECK(hipGetLastError());
    } else {                             // run-time specialized k_all_<name> (same arguments)
      int* wl = c->worklist + 2;
      int* efc = c->mirror.efc_count;
      void* args[] = {&c->mirror, &B, &qpos, &qvel, &qacc, &qfrc, &status, &wl, &cnt, &nxt,
                      &efc, (void*)&range};
      HIPCHECK(hipModuleLaunchKernel(c->rt_fn, grid.x, 1, 1, 64, 1, 1, 0, c->stream, args,
                                     nullptr));
    }
    if (flags & kFlagDeferRows) {
      // mjhip_inverseFDBatch: the work-list this launch filled is served after the next
      // launch, which appends to the same counter (the parity is not flipped)
      return MJHIP_OK;
    }
    if (c->spatial) {                    // spatial tendons and all of mj_passive
      hipLaunchKernelGGL(k_tendon_after, grid, block, 0, c->stream, c->dmodel, c->mirror, B);
    } else if (mjh::hasFluid(c->dmodel)) {   // fluid forces into qfrc_passive
      hipLaunchKernelGGL(k_fluid_after, grid, block, 0, c->stream, c->dmodel, c->mirror, B);
    }
    if (discrete) {                      // mj_discreteAcc and its RNE before the constraints
      hipLaunchKernelGGL(k_discrete_before, grid, block, 0, c->stream, c->dmodel, c->mirror, B,
                         mjh_needTrnAfter(&c->hmodel));
    }
    const int* wl = c->worklist + 2;
    if (fused && c->coop && c->fast->cmode) {   // cooperative lanes per instance
      const bool contact = c->con_cap > 0, list = c->fast->cmode == 1;
#define MJHIP_LAUNCH_COOP(G, C, L, X)                                                         \
      do {                                                                                    \
        c->con_kernel = "k_constraint_coop<" #G ", " #C ", " #L ", " #X ">";                \
        hipLaunchKernelGGL((k_constraint_coop<G, C, L, X>), dim3(coopGrid(B, G, L)),          \
                           dim3(64), coopLdsBytes(c->dmodel, G, c->efc_cap, c->boxpair,       \
                                                  c->npair, c->con_cap),                      \
                           c->stream,                                                         \
                           c->dmodel, c->mirror, B, wl,                                       \
                           (const int*)cnt, c->pairs, c->cparams, c->masks, c->npair, qfrc,  \
                           status, nullptr);                                                  \
      } while (0)
      if (contact && c->boxpair) {       // the box-box path is compiled in only here
        if (list) MJHIP_LAUNCH_COOP(16, true, true, true);
        else MJHIP_LAUNCH_COOP(16, true, false, true);
      } else if (contact) {
        if (list) MJHIP_LAUNCH_COOP(16, true, true, false);
        else if (c->coop == 8) MJHIP_LAUNCH_COOP(8, true, false, false);
        else if (c->coop == 32) MJHIP_LAUNCH_COOP(32, true, false, false);
        else MJHIP_LAUNCH_COOP(16, true, false, false);
      } else {
        if (list) MJHIP_LAUNCH_COOP(16, false, true, false);
        else MJHIP_LAUNCH_COOP(16, false, false, false);
      }
#undef MJHIP_LAUNCH_COOP
    } else {
#define MJHIP_LAUNCH_CON(C, F, L)                                                             \
    do {                                                                                      \
      c->con_kernel = "k_constraint<" #C ", " #F ", " #L ">";                               \
      hipLaunchKernelGGL((k_constraint<C, F, L>), grid, block,                                \
                         ((C && F) ? mjh::gstageBytes(c->dmodel) : 0) +                       \
                         ((!L && qfrc) ? 64u*sizeof(double)*c->dmodel.nv : 0), c->stream,    \
                         c->dmodel, c->mirror, B, wl, (const int*)cnt, qfrc, status);         \
    } while (0)
    if (c->fast->cmode == 2) {          // contacts or friction loss: every instance
      if (c->con_cap > 0) {
        if (fused) MJHIP_LAUNCH_CON(true, true, false); else MJHIP_LAUNCH_CON(true, false, false);
      } else {
        if (fused) MJHIP_LAUNCH_CON(false, true, false);
        else MJHIP_LAUNCH_CON(false, false, false);
      }
    } else if (c->fast->cmode == 1) {   // limit-active instances (k_pos's work-list)
      if (fused) MJHIP_LAUNCH_CON(false, true, true); else MJHIP_LAUNCH_CON(false, false, true);
    }
#undef MJHIP_LAUNCH_CON
    }
    HIPCHECK(hipGetLastError());
    return finish_fast(c, B, grid, block, skipsensor, status, discrete);
  }
  // mj_inverseSkip(POS / VEL) on the straight-line kernels: the bare pipeline (no passes
  // after the generated kernels) of a model whose rows serve only limit-active instances
  const char* noskip = getenv("MJHIP_SKIP_GENERIC");
  if ((skipstage == mjhipSTAGE_POS || skipstage == mjhipSTAGE_VEL) && c->fast &&
      c->fast->launch_skip && !(flags & MJHIP_FLAG_GENERIC) && !c->spatial &&
      !mjh::hasFluid(c->hmodel) && !mjh::hasDiscrete(c->hmodel) &&
      !mjh_needTrnAfter(&c->hmodel) && !(c->hmodel.opt.enableflags & mjhipENBL_ENERGY) &&
      (skipsensor || !c->hmodel.nsensor || (c->hmodel.opt.disableflags & mjhipDSBL_SENSOR)) &&
      !(noskip && noskip[0] == '1')) {
    // row-major inputs into the mirror, as k_inverse copies them: the remaining stages read
    // qpos (springs) and qvel (mj_rne's cdof_dot * qvel) even when their own stage is skipped
    const int nq = c->hmodel.nq, nv = c->hmodel.nv;
    if (qpos) {
      hipLaunchKernelGGL(k_to_mirror, dim3(((long)B*nq + 255)/256), dim3(256), 0, c->stream,
                         qpos, c->mirror.qpos, B, nq);
    }
    if (qvel) {
      hipLaunchKernelGGL(k_to_mirror, dim3(((long)B*nv + 255)/256), dim3(256), 0, c->stream,
                         qvel, c->mirror.qvel, B, nv);
    }
    if (qacc) {
      hipLaunchKernelGGL(k_to_mirror, dim3(((long)B*nv + 255)/256), dim3(256), 0, c->stream,
                         qacc, c->mirror.qacc, B, nv);
    }
    c->last_path = 2;
    c->fast->launch_skip(c->stream, c->mirror, B, skipstage, qfrc, status, c->mirror.efc_count);
    HIPCHECK(hipGetLastError());
    if (c->fast->cmode) {                // work-list rows, or every instance (contacts)
      hipLaunchKernelGGL(k_skip_rows, grid, block, 0, c->stream, c->dmodel, c->mirror, B,
                         skipstage, qfrc, (int)(c->fast->cmode == 2));
      HIPCHECK(hipGetLastError());
    }
    if (status) {
      hipLaunchKernelGGL(k_check, grid, block, 0, c->stream, c->dmodel, c->mirror, B, status,
                         skipstage);
      HIPCHECK(hipGetLastError());
    }
    return MJHIP_OK;
  }
#define MJHIP_LAUNCH_K(SK, C, F)                                                              \
  hipLaunchKernelGGL((k_inverse<SK, C, F>), grid, block,                                      \
                     (C && F) ? mjh::gstageBytes(c->dmodel) : 0, c->stream, c->dmodel,        \
                     c->mirror, B, qpos, qvel, qacc, qfrc, status, skipsensor)
#define MJHIP_LAUNCH_GENERIC(SK)                                                              \
  if (c->con_cap > 0) {                                                                       \
    MJHIP_LAUNCH_K(SK, true, false);                                                          \
  } else {                                                                                    \
    MJHIP_LAUNCH_K(SK, false, false);                                                         \
  }
  switch (skipstage) {
  case mjhipSTAGE_NONE:
    if (mjh::fusedOk(c->dmodel, mjhipSTAGE_NONE)) {
      if (c->con_cap > 0) MJHIP_LAUNCH_K(0, true, true); else MJHIP_LAUNCH_K(0, false, true);
    } else {
      MJHIP_LAUNCH_GENERIC(0)
    }
    break;
  case mjhipSTAGE_POS:
    MJHIP_LAUNCH_GENERIC(1)
    break;
  case mjhipSTAGE_VEL:
    MJHIP_LAUNCH_GENERIC(2)
    break;
  default:
    set_error("skipstage must be mjSTAGE_NONE, mjSTAGE_POS or mjSTAGE_VEL");
    return MJHIP_ERR_ARG;
  }
#undef MJHIP_LAUNCH_GENERIC
#undef MJHIP_LAUNCH_K
  HIPCHECK(hipGetLastError());
  return MJHIP_OK;
}

//---------------------------------- per-stage timers ------------------------------------------

// point every copy of mjh_tbuf (this unit's, the generated kernels' and the run-time code
// object's) at p; blocking copies, after the stream's earlier work
static int timers_attach(mjhipContext* c, unsigned long long* p) {
  HIPCHECK(hipStreamSynchronize(c->stream));
  HIPCHECK(hipMemcpyToSymbol(HIP_SYMBOL(mjh_tbuf), &p, sizeof(p)));
  if (mjhip_genSetTimerBuf(p) || mjhip_genExactSetTimerBuf(p) ||
      mjhip_setTimerBufConstraint(p) ||
      mjhip_setTimerBufInverse(p)) {
    set_error("setting the kernel units' timer pointers failed");
    return MJHIP_ERR_HIP;
  }
  if (c->rt_tbuf) HIPCHECK(hipMemcpyHtoD(c->rt_tbuf, &p, sizeof(p)));
  return MJHIP_OK;
}

// point every mjh_tbuf copy back at null (after the stream's earlier work), so that no kernel
// adds into an accumulator that is about to be freed; the caller frees it only on success
static int timers_detach(mjhipContext* c) {
  const int rc = timers_attach(c, nullptr);
  if (g_timed_ctx == c) g_timed_ctx = nullptr;
  return rc;
}

// fold one call's phase-mark sums (engine_device.h MJH_PHASE: slots and wave counts) into
// the reference's timer slots: mean wave time per stage, 100 MHz ticks -> milliseconds
static void timers_fold(mjhipContext* c, const unsigned long long* t, float call_ms) {
  auto span = [&](int a, int b, int n) {
    return t[n] ? (double)(long long)(t[b] - t[a]) / (double)t[n] / 1e5 : 0.0;
  };
  double kin = 0, inertia = 0, col = 0, make = 0, vel = 0, con = 0;
  if (t[24]) {                             // generic k_inverse, marks 0-9
    kin += span(0, 1, 24) + span(1, 2, 24) + span(5, 6, 24);
    inertia += span(2, 3, 24);
    col += span(3, 4, 24);
    make += span(4, 5, 24);
    vel += span(6, 7, 24);
    con += span(7, 8, 24);
  }
  if (t[27]) {                             // straight-line k_all, marks 19-22
    kin += span(19, 20, 27);
    inertia += span(20, 21, 27);
    vel += span(21, 22, 27);
  }
  if (t[25]) {                             // one-lane k_constraint, marks 10-13
    col += span(10, 11, 25);
    make += span(11, 12, 25);
    con += span(12, 13, 25);
  }
  if (t[26]) {                             // k_constraint_coop, marks 14, 15, (18,) 16, 17
    col += span(14, 15, 26);
    make += t[18] ? span(15, 18, 26) + span(18, 16, 26) : span(15, 16, 26);
    con += span(16, 17, 26);
  }
  auto add = [&](int slot, double ms) {
    c->timer[slot].duration += ms;
    c->timer[slot].number += 1;
  };
  add(mjhipTIMER_INVERSE, call_ms);
  add(mjhipTIMER_POSITION, kin + inertia + col + make);
  add(mjhipTIMER_POS_KINEMATICS, kin);
  add(mjhipTIMER_POS_INERTIA, inertia);
  add(mjhipTIMER_POS_COLLISION, col);
  add(mjhipTIMER_POS_MAKE, make);
  add(mjhipTIMER_VELOCITY, vel);
  add(mjhipTIMER_CONSTRAINT, con);
}

MJHIP_API int mjhip_contextTimers(mjhipContext* c, int enable) {
  if (!c) {
    set_error("mjhip_contextTimers: null context");
    return MJHIP_ERR_ARG;
  }
  HIPCHECK(hipSetDevice(c->device));
  if (!enable) {
    if (c->tbuf) {
      if (const int rc = timers_detach(c)) return rc;   // a unit may still point at it
      HIPCHECK(hipFree(c->tbuf));
      c->tbuf = nullptr;
    }
    if (g_timed_ctx == c) g_timed_ctx = nullptr;
    return MJHIP_OK;
  }
  if (g_timed_ctx && g_timed_ctx != c) {
    set_error("mjhip_contextTimers: another context of this process is being timed");
    return MJHIP_ERR_ARG;
  }
  if (!c->tbuf) {
    unsigned long long* buf = nullptr;
    HIPCHECK(hipMalloc((void**)&buf, MJH_TSLOTS * sizeof(unsigned long long)));
    if (hipMemset(buf, 0, MJH_TSLOTS * sizeof(unsigned long long)) != hipSuccess) {
      hipFree(buf);
      set_error("mjhip_contextTimers: hipMemset failed");
      return MJHIP_ERR_HIP;
    }
    c->tbuf = buf;
  }
  if (!c->tev0) HIPCHECK(hipEventCreate(&c->tev0));
  if (!c->tev1) HIPCHECK(hipEventCreate(&c->tev1));
  g_timed_ctx = c;                         // only once everything it needs exists
  return MJHIP_OK;
}

MJHIP_API int mjhip_timerRead(mjhipContext* c, mjhipTimerStat* out, int reset) {
  if (!c || !out) {
    set_error("mjhip_timerRead: bad argument");
    return MJHIP_ERR_ARG;
  }
  memcpy(out, c->timer, sizeof(c->timer));
  if (reset) memset(c->timer, 0, sizeof(c->timer));
  return MJHIP_OK;
}

MJHIP_API int mjhip_inverseBatch(mjhipContext* c, int B, const mjtNum* qpos,
                                 const mjtNum* qvel, const mjtNum* qacc, mjtNum* qfrc_inverse,
                                 int skipstage, int skipsensor, int flags, int* status) {
  if (!c || B < 0) {
    set_error("mjhip_inverseBatch: bad argument");
    return MJHIP_ERR_ARG;
  }
  if (B > c->capacity) {
    set_error("batch %d exceeds context capacity %d", B, c->capacity);
    return MJHIP_ERR_CAPACITY;
  }
  if (B == 0) return MJHIP_OK;
  HIPCHECK(hipSetDevice(c->device));
  const mjhipModel& m = c->hmodel;
  const bool dev = flags & MJHIP_FLAG_DEVICE_PTRS;
  const bool mirror_in = flags & MJHIP_FLAG_MIRROR_INPUT;
  const double *dq = nullptr, *dv = nullptr, *da = nullptr;
  double* dqfrc = nullptr;
  double* sq = c->stage;
  double* sv = sq + (size_t)c->capacity*m.nq;
  double* sa = sv + (size_t)c->capacity*m.nv;
  double* sf = sa + (size_t)c->capacity*m.nv;
  if (!mirror_in) {
    if (!qpos || !qvel || !qacc) {
      set_error("mjhip_inverseBatch: qpos/qvel/qacc required without MJHIP_FLAG_MIRROR_INPUT");
      return MJHIP_ERR_ARG;
    }
    if (dev) {
      dq = qpos; dv = qvel; da = qacc;
    } else {
      HIPCHECK(hipMemcpyAsync(sq, qpos, sizeof(double)*(size_t)B*m.nq, hipMemcpyHostToDevice,
                              c->stream));
      HIPCHECK(hipMemcpyAsync(sv, qvel, sizeof(double)*(size_t)B*m.nv, hipMemcpyHostToDevice,
                              c->stream));
      HIPCHECK(hipMemcpyAsync(sa, qacc, sizeof(double)*(size_t)B*m.nv, hipMemcpyHostToDevice,
                              c->stream));
      dq = sq; dv = sv; da = sa;
    }
  }
  if (qfrc_inverse) dqfrc = dev ? qfrc_inverse : sf;
  // per-instance statuses only when the caller can see them (status array, or the host path's
  // return code): a device-pointer call without them skips the input checks entirely
  const bool want_status = status || !dev;
  const bool timed = c->tbuf != nullptr;
  if (timed) {
    int trc = timers_attach(c, c->tbuf);
    if (trc) {
      timers_attach(c, nullptr);
      return trc;
    }
    HIPCHECK(hipEventRecord(c->tev0, c->stream));
  }
  int rc = launch_inverse(c, B, dq, dv, da, dqfrc, skipstage, want_status ? c->status : nullptr,
                          flags, skipsensor);
  if (timed) {
    HIPCHECK(hipEventRecord(c->tev1, c->stream));
    const int arc = timers_attach(c, nullptr);   // synchronizes the stream first
    if (rc) return rc;
    if (arc) return arc;
    unsigned long long t[MJH_TSLOTS];
    float call_ms = 0;
    HIPCHECK(hipMemcpy(t, c->tbuf, sizeof(t), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemset(c->tbuf, 0, sizeof(t)));
    HIPCHECK(hipEventElapsedTime(&call_ms, c->tev0, c->tev1));
    for (int k = 0; k < MJH_TSLOTS; k++) c->traw[k] += t[k];
    timers_fold(c, t, call_ms);
  }
  if (rc) return rc;
  if (qfrc_inverse && !dev) {
    HIPCHECK(hipMemcpyAsync(qfrc_inverse, sf, sizeof(double)*(size_t)B*m.nv,
                            hipMemcpyDeviceToHost, c->stream));
  }
  int anybad = 0;
  if (want_status) {
    std::vector<int> st(B);
    HIPCHECK(hipMemcpyAsync(st.data(), c->status, sizeof(int)*(size_t)B, hipMemcpyDeviceToHost,
                            c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < B; i++) anybad |= st[i];
    if (status) memcpy(status, st.data(), sizeof(int)*(size_t)B);
  }
  return anybad ? MJHIP_ERR_INSTANCE : MJHIP_OK;
}

MJHIP_API int mjhip_forwardBatch(mjhipContext* c, int B, const mjtNum* qpos, const mjtNum* qvel,
                                 const mjtNum* ctrl, mjtNum* qacc, int flags, int* status) {
  if (!c || B < 0) {
    set_error("mjhip_forwardBatch: bad argument");
    return MJHIP_ERR_ARG;
  }
  if (B > c->capacity) {
    set_error("batch %d exceeds context capacity %d", B, c->capacity);
    return MJHIP_ERR_CAPACITY;
  }
  const mjhipModel& m = c->hmodel;
  for (int i = 0; i < m.nu; i++) {
    if ((m.actuator_gaintype[i] != mjhipGAIN_FIXED && m.actuator_gaintype[i] != mjhipGAIN_AFFINE) ||
        (m.actuator_biastype[i] != mjhipBIAS_NONE && m.actuator_biastype[i] != mjhipBIAS_AFFINE) ||
        m.actuator_dyntype[i] != mjhipDYN_NONE) {
      set_error("mjhip_forwardBatch: muscle/user gain or bias, or actuator dynamics (act), "
                "is not supported");
      return MJHIP_ERR_MODEL;
    }
  }
  if (B == 0) return MJHIP_OK;
  HIPCHECK(hipSetDevice(c->device));
  const bool dev = flags & MJHIP_FLAG_DEVICE_PTRS;
  const bool mirror_in = flags & MJHIP_FLAG_MIRROR_INPUT;
  const double *dq = nullptr, *dv = nullptr, *dc = nullptr;
  double* sq = c->stage;
  double* sv = sq + (size_t)c->capacity*m.nq;
  double* sa = sv + (size_t)c->capacity*m.nv;
  double* sc = sa + 2*(size_t)c->capacity*m.nv;
  if (!mirror_in) {
    if (!qpos || !qvel) {
      set_error("mjhip_forwardBatch: qpos/qvel required without MJHIP_FLAG_MIRROR_INPUT");
      return MJHIP_ERR_ARG;
    }
    if (dev) {
      dq = qpos; dv = qvel; dc = ctrl;
    } else {
      HIPCHECK(hipMemcpyAsync(sq, qpos, sizeof(double)*(size_t)B*m.nq, hipMemcpyHostToDevice,
                              c->stream));
      HIPCHECK(hipMemcpyAsync(sv, qvel, sizeof(double)*(size_t)B*m.nv, hipMemcpyHostToDevice,
                              c->stream));
      if (ctrl && m.nu) {
        HIPCHECK(hipMemcpyAsync(sc, ctrl, sizeof(double)*(size_t)B*m.nu, hipMemcpyHostToDevice,
                                c->stream));
      }
      dq = sq; dv = sv; dc = (ctrl && m.nu) ? sc : nullptr;
    }
  }
  double* dqacc = qacc ? (dev ? qacc : sa) : nullptr;
  dim3 grid((B + 63) / 64), block(64);
  if (c->con_cap > 0) {
    hipLaunchKernelGGL(k_forward<true>, grid, block, 0, c->stream, c->dmodel, c->mirror, B, dq,
                       dv, dc, dqacc, c->status);
  } else {
    hipLaunchKernelGGL(k_forward<false>, grid, block, 0, c->stream, c->dmodel, c->mirror, B, dq,
                       dv, dc, dqacc, c->status);
  }
  HIPCHECK(hipGetLastError());
  if (qacc && !dev) {
    HIPCHECK(hipMemcpyAsync(qacc, sa, sizeof(double)*(size_t)B*m.nv, hipMemcpyDeviceToHost,
                            c->stream));
  }
  int anybad = 0;
  if (status || !dev) {
    std::vector<int> st(B);
    HIPCHECK(hipMemcpyAsync(st.data(), c->status, sizeof(int)*(size_t)B, hipMemcpyDeviceToHost,
                            c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < B; i++) anybad |= st[i];
    if (status) memcpy(status, st.data(), sizeof(int)*(size_t)B);
  }
  return anybad ? MJHIP_ERR_INSTANCE : MJHIP_OK;
}

MJHIP_API int mjhip_statusDownload(mjhipContext* c, int first, int count, int* dst) {
  if (!c || first < 0 || count < 0 || first + count > c->capacity || !dst) return MJHIP_ERR_ARG;
  HIPCHECK(hipSetDevice(c->device));
  HIPCHECK(hipMemcpyAsync(dst, c->status + first, sizeof(int)*(size_t)count,
                          hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  return MJHIP_OK;
}

// element k of instance i (counted from the first fetched block) of an S-element field at
// tmp[base + k*step]: lane-interleaved (F[(blk*S + k)*64 + lane]) or instance-contiguous
// (F[(blk*64 + lane)*S + k], the XSCC / XSIC fields)
static void blockIndex(int i, int S, bool contig, size_t* base, size_t* step) {
  if (contig) {
    *base = (size_t)i * S;
    *step = 1;
  } else {
    *base = (size_t)(i / 64) * S * 64 + (i & 63);
    *step = 64;
  }
}

static int find_field(mjhipContext* c, const char* field, double** ptr, int* S) {
  auto it = c->fields.find(field);
  if (it == c->fields.end()) {
    set_error("unknown mirror field '%s'", field);
    return MJHIP_ERR_ARG;
  }
  *ptr = it->second.first;
  *S = it->second.second;
  return MJHIP_OK;
}

MJHIP_API void* mjhip_mirrorDevicePtr(mjhipContext* c, const char* field) {
  double* p;
  int S;
  if (!c || find_field(c, field, &p, &S)) return nullptr;
  return p;
}

// int scratch fields (constraint row types/ids/states, counts, contact geoms/dims), one
// instance-major row of `S` ints per instance
MJHIP_API int mjhip_mirrorDownloadInt(mjhipContext* c, const char* field, int first, int count,
                                      int* dst) {
  if (!c || !field || !dst || first < 0 || count < 0 || first + count > c->capacity) {
    return MJHIP_ERR_ARG;
  }
  auto it = c->ifields.find(field);
  if (it == c->ifields.end()) {
    set_error("unknown int mirror field '%s'", field);
    return MJHIP_ERR_ARG;
  }
  int* p = it->second.first;
  int S = it->second.second;
  if (!count || !S) return MJHIP_OK;
  HIPCHECK(hipSetDevice(c->device));
  int b0 = first / 64, b1 = (first + count + 63) / 64;
  std::vector<int> tmp((size_t)(b1 - b0) * S * 64);
  HIPCHECK(hipMemcpyAsync(tmp.data(), p + (size_t)b0*S*64, tmp.size()*sizeof(int),
                          hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  const bool ct = c->contig.count(field) > 0;
  for (int i = 0; i < count; i++) {
    int inst = first + i;
    size_t base, step;
    blockIndex(inst - b0*64, S, ct, &base, &step);
    for (int k = 0; k < S; k++) dst[(size_t)i*S + k] = tmp[base + (size_t)k*step];
  }
  return MJHIP_OK;
}

MJHIP_API int mjhip_mirrorFieldSize(const mjhipContext* c, const char* field) {
  if (!c || !field) return -1;
  auto it = c->fields.find(field);
  return it == c->fields.end() ? -1 : it->second.second;
}

MJHIP_API int mjhip_fieldSizeInt(const mjhipContext* c, const char* field) {
  if (!c || !field) return -1;
  auto it = c->ifields.find(field);
  return it == c->ifields.end() ? -1 : it->second.second;
}

// host transfers of whole 64-instance blocks, reordered on the host
MJHIP_API int mjhip_mirrorDownload(mjhipContext* c, const char* field, int first, int count,
                                   mjtNum* dst) {
  double* p;
  int S;
  if (!c || !dst || first < 0 || count < 0 || first + count > c->capacity) return MJHIP_ERR_ARG;
  if (int rc = find_field(c, field, &p, &S)) return rc;
  if (!count || !S) return MJHIP_OK;
  HIPCHECK(hipSetDevice(c->device));
  int b0 = first / 64, b1 = (first + count + 63) / 64;
  std::vector<double> tmp((size_t)(b1 - b0) * S * 64);
  HIPCHECK(hipMemcpyAsync(tmp.data(), p + (size_t)b0*S*64, tmp.size()*sizeof(double),
                          hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  const bool ct = c->contig.count(field) > 0;
  for (int i = 0; i < count; i++) {
    int inst = first + i;
    size_t base, step;
    blockIndex(inst - b0*64, S, ct, &base, &step);
    for (int k = 0; k < S; k++) dst[(size_t)i*S + k] = tmp[base + (size_t)k*step];
  }
  return MJHIP_OK;
}

MJHIP_API int mjhip_mirrorUpload(mjhipContext* c, const char* field, int first, int count,
                                 const mjtNum* src) {
  double* p;
  int S;
  if (!c || !src || first < 0 || count < 0 || first + count > c->capacity) return MJHIP_ERR_ARG;
  if (int rc = find_field(c, field, &p, &S)) return rc;
  if (!count || !S) return MJHIP_OK;
  HIPCHECK(hipSetDevice(c->device));
  int b0 = first / 64, b1 = (first + count + 63) / 64;
  std::vector<double> tmp((size_t)(b1 - b0) * S * 64);
  HIPCHECK(hipMemcpyAsync(tmp.data(), p + (size_t)b0*S*64, tmp.size()*sizeof(double),
                          hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  const bool ct = c->contig.count(field) > 0;
  for (int i = 0; i < count; i++) {
    int inst = first + i;
    size_t base, step;
    blockIndex(inst - b0*64, S, ct, &base, &step);
    for (int k = 0; k < S; k++) tmp[base + (size_t)k*step] = src[(size_t)i*S + k];
  }
  HIPCHECK(hipMemcpyAsync(p + (size_t)b0*S*64, tmp.data(), tmp.size()*sizeof(double),
                          hipMemcpyHostToDevice, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  return MJHIP_OK;
}

MJHIP_API int mjhip_timeInverseKernel(mjhipContext* c, int B, int reps, int skipstage,
                                      int flags, float* ms) {
  if (!c || B <= 0 || B > c->capacity || reps <= 0 || !ms) return MJHIP_ERR_ARG;
  HIPCHECK(hipSetDevice(c->device));
  HIPCHECK(hipEventRecord(c->ev0, c->stream));
  for (int r = 0; r < reps; r++) {
    int rc = launch_inverse(c, B, nullptr, nullptr, nullptr, nullptr, skipstage, nullptr,
                            flags);
    if (rc) return rc;
  }
  HIPCHECK(hipEventRecord(c->ev1, c->stream));
  HIPCHECK(hipEventSynchronize(c->ev1));
  float t = 0;
  HIPCHECK(hipEventElapsedTime(&t, c->ev0, c->ev1));
  *ms = t / reps;
  return MJHIP_OK;
}

// actuator subset of the device mj_fwdActuation (mjh::fwdActuation): fixed/affine gain,
// none/affine bias, no activation dynamics
static const char* actuation_unsupported(const mjhipModel& m) {
  for (int i = 0; i < m.nu; i++) {
    if ((m.actuator_gaintype[i] != mjhipGAIN_FIXED && m.actuator_gaintype[i] != mjhipGAIN_AFFINE) ||
        (m.actuator_biastype[i] != mjhipBIAS_NONE && m.actuator_biastype[i] != mjhipBIAS_AFFINE) ||
        m.actuator_dyntype[i] != mjhipDYN_NONE) {
      return "muscle/user gain or bias, or actuator dynamics (act)";
    }
  }
  return nullptr;
}

MJHIP_API int mjhip_inverseFDBatchEx(mjhipContext* c, int B, const mjtNum* qpos,
                                     const mjtNum* qvel, const mjtNum* qacc, const mjtNum* ctrl,
                                     mjtNum eps, int flg_actuation, mjtNum* DfDq, mjtNum* DfDv,
                                     mjtNum* DfDa, mjtNum* DsDq, mjtNum* DsDv, mjtNum* DsDa,
                                     mjtNum* DmDq, int flags) {
  if (!c || B <= 0 || !qpos || !qvel || !qacc || (flg_actuation && c->hmodel.nu && !ctrl)) {
    set_error("mjhip_inverseFDBatch: bad argument");
    return MJHIP_ERR_ARG;
  }
  const mjhipModel& m = c->hmodel;
  const int nv = m.nv, P = 3*nv + 1;
  if (m.opt.integrator == mjhipINT_RK4) {       // engine_derivative_fd.c:619-621
    set_error("mjd_inverseFD: RK4 integrator is not supported");
    return MJHIP_ERR_MODEL;
  }
  if (m.nmocap) {
    set_error("mjhip_inverseFDBatch: mocap poses per base state are not an input of the "
              "batched FD API");
    return MJHIP_ERR_MODEL;
  }
  if (flg_actuation) {
    if (const char* why = actuation_unsupported(m)) {
      set_error("mjhip_inverseFDBatch(flg_actuation): %s is not supported", why);
      return MJHIP_ERR_MODEL;
    }
  }
  if ((long)B*P > c->capacity) {
    set_error("FD batch needs %ld instances, context capacity %d", (long)B*P, c->capacity);
    return MJHIP_ERR_CAPACITY;
  }
  HIPCHECK(hipSetDevice(c->device));
  const bool dev = flags & MJHIP_FLAG_DEVICE_PTRS;
  const double *dq = qpos, *dv = qvel, *da = qacc, *dc = flg_actuation ? ctrl : nullptr;
  // per-call device buffers of the host-array form (ctrl, the Jacobians); freed on every
  // return path, after the stream has finished with them (the device-pointer form has none
  // and returns without waiting for the device)
  struct Scratch {
    mjhipContext* c;
    std::vector<double*> p;
    ~Scratch() {
      if (p.empty()) return;
      hipStreamSynchronize(c->stream);
      for (double* d : p) hipFree(d);
    }
    double* alloc(size_t n) {
      double* d = nullptr;
      if (hipMalloc((void**)&d, (n ? n : 1)*sizeof(double)) != hipSuccess) return nullptr;
      p.push_back(d);
      return d;
    }
  } tmp{c, {}};
#define FDCHECK(expr, what)                                                                   \
  do {                                                                                        \
    if ((expr) != hipSuccess) {                                                               \
      set_error("mjhip_inverseFDBatch: %s failed", what);                                    \
      return MJHIP_ERR_HIP;                                                                   \
    }                                                                                         \
  } while (0)
  if (!dev) {
    double* sq = c->stage;
    double* sv = sq + (size_t)c->capacity*m.nq;
    double* sa = sv + (size_t)c->capacity*m.nv;
    FDCHECK(hipMemcpyAsync(sq, qpos, sizeof(double)*(size_t)B*m.nq, hipMemcpyHostToDevice,
                           c->stream), "qpos upload");
    FDCHECK(hipMemcpyAsync(sv, qvel, sizeof(double)*(size_t)B*nv, hipMemcpyHostToDevice,
                           c->stream), "qvel upload");
    FDCHECK(hipMemcpyAsync(sa, qacc, sizeof(double)*(size_t)B*nv, hipMemcpyHostToDevice,
                           c->stream), "qacc upload");
    dq = sq; dv = sv; da = sa;
    if (dc && m.nu) {
      double* sc = tmp.alloc((size_t)B*m.nu);
      if (!sc) { set_error("hipMalloc(ctrl) failed"); return MJHIP_ERR_HIP; }
      FDCHECK(hipMemcpyAsync(sc, ctrl, sizeof(double)*(size_t)B*m.nu, hipMemcpyHostToDevice,
                             c->stream), "ctrl upload");
      dc = sc;
    }
  }
  long ninst = (long)B*P;
  // sensors are skipped when no sensor derivative is asked for (derivative_fd.c:628)
  const int skipsensor = !DsDq && !DsDv && !DsDa;
  // Stage skipping as the reference's loop does (engine_derivative_fd.c:646-699): the qvel
  // perturbations run mj_inverseSkip(mjSTAGE_POS), only the generated va stage over their
  // centre's position-stage outputs, and the qacc ones mjSTAGE_VEL, the acceleration stage
  // alone over the centre's position and velocity stages (layout 2, k_fdskip; layout 1 runs
  // both kinds on the va stage, k_vaskip). Skipped stages would see unchanged inputs: layout 1
  // equals the full pipeline bit for bit; layout 2 is the same arithmetic in a differently
  // shaped kernel, where the compiler's multiply-add contraction can round a term differently
  // (a few ulp of qfrc_inverse). Taken only where the straight-line kernel
  // is the whole pipeline (no post passes, sensors or actuation terms) and the
  // position-stage block ends on a wave boundary.
  const long nA = (long)B*(nv + 1), nQ = (long)B*nv;
  const char* noskip = getenv("MJHIP_FD_NOSKIP");
  const char* accskip = getenv("MJHIP_FD_ACCSKIP");
  int layout = c->fast && c->fast->launch_vaskip && !(flags & MJHIP_FLAG_GENERIC) &&
               skipsensor && !flg_actuation && !c->spatial && !mjh::hasFluid(c->hmodel) &&
               !mjh::hasDiscrete(c->hmodel) && !mjh_needTrnAfter(&c->hmodel) &&
               !(m.opt.enableflags & mjhipENBL_ENERGY) && nA % 64 == 0 &&
               !(noskip && noskip[0] == '1') && !(flags & kFlagFDFull);
  // layout 2 on request (MJHIP_FD_ACCSKIP=1), when the two perturbation blocks are whole waves
  // each: not the default, as it measured no faster (k_fdskip 62-64 us against k_vaskip's
  // 56 us over the same 55,296 instances)
  if (layout && c->fast->launch_fdskip && nQ % 64 == 0 && accskip && accskip[0] == '1') layout = 2;
  int rc = MJHIP_OK;
  // a skip layout's perturbed instances store only what a later kernel of this call reads
  // (codegen.FD_KEEP): instance blocks past the centres' drop the rest, as the launches below
  // see through the mirror; restored on every return path
  struct ElideGuard {
    Mirror* mr;
    ~ElideGuard() { mr->fd_elide = 0; mr->full_blk = 0; }
  } elide_guard{&c->mirror};
  if (layout) {
    c->mirror.fd_elide = 1;
    c->mirror.full_blk = (B + 63) / 64;
  }
  // with a skip layout only the position-stage block is expanded: the skip kernels read their
  // centre's inputs and perturb them in registers (the fall-back expands the rest, below)
  const long nexp = layout ? nA : ninst;
  hipLaunchKernelGGL(k_fd_expand, dim3((unsigned)((nexp + 63)/64)), dim3(64*kExpandWaves), 0,
                     c->stream, c->dmodel, c->mirror, B, dq, dv, da, (m.nu ? dc : nullptr),
                     eps, layout, layout ? c->fdflag : nullptr, (long)0, nexp, 0);
  FDCHECK(hipGetLastError(), "k_fd_expand launch");
  // MJHIP_FD_FUSED=1: layout 1 in one launch (k_fdall) -- measured slower than the two
  // launches (config 5: 4.81M against 5.13M Jacobian sets/s on one box), kept for
  // the A/B
  const char* fusedfd = getenv("MJHIP_FD_FUSED");
  if (layout == 1 && c->fast->launch_fdall && c->fast->launch && fusedfd && fusedfd[0] == '1') {
    // one launch (k_fdall): the position-stage instances' full pipeline on the first blocks,
    // the qvel/qacc perturbations' va stage beside them, each skip wave once its centres'
    // position stage is out (a work-list model's rows are served after the fall-back, as
    // below; a model without rows hands the work-list counters on as launch_inverse does)
    if (!c->fdflags) {
      const size_t n = (size_t)c->capacity / 64 + 1;
      FDCHECK(hipMalloc((void**)&c->fdflags, n*sizeof(int)), "hipMalloc(FD flags)");
      FDCHECK(hipMemset(c->fdflags, 0, n*sizeof(int)), "hipMemset(FD flags)");
      c->fd_epoch = 0;
    }
    if (++c->fd_epoch == 0x7fffffff) {     // flags from 2^31 calls ago could match again
      FDCHECK(hipMemsetAsync(c->fdflags, 0, ((size_t)c->capacity / 64 + 1)*sizeof(int),
                             c->stream), "hipMemset(FD flags)");
      c->fd_epoch = 1;
    }
    int* cnt = c->worklist + c->wl_parity;
    int* nxt = c->worklist + (c->wl_parity ^ 1);
    c->last_path = 1;
    c->fast->launch_fdall(c->stream, c->mirror, (int)nA, (int)ninst, 2*nv, eps, c->worklist + 2,
                          cnt, nxt, c->mirror.efc_count, c->fdflag, c->fdflags, c->fd_epoch);
    FDCHECK(hipGetLastError(), "k_fdall launch");
    if (c->fast->cmode != 1) {
      c->wl_last = c->wl_parity;
      c->wl_parity ^= 1;
    }
  } else if (layout) {
    // the nv+1 position-stage instances of every base state: the full pipeline (a work-list
    // model's rows are served once, after the fall-back below has added its own)
    const bool defer = c->fast->cmode == 1 && c->fast->launch;
    rc = launch_inverse(c, (int)nA, nullptr, nullptr, nullptr, nullptr, mjhipSTAGE_NONE,
                        nullptr, defer ? kFlagDeferRows : 0, skipsensor);
    if (rc) return rc;
    if (layout == 2) {
      // the nv qacc perturbations: the acceleration stage over their centre's position and
      // velocity stages; the nv qvel ones: the va stage over their centre's position stage
      c->fast->launch_fdskip(c->stream, c->mirror, (int)ninst, (int)nA, nv, 1,
                             c->mirror.efc_count, c->fdflag, eps);
    } else {
      // the 2nv qvel/qacc perturbations: the va stage over their centre's position stage
      c->fast->launch_vaskip(c->stream, c->mirror, (int)ninst, (int)nA, 2*nv, 1,
                             c->mirror.efc_count, c->fdflag, eps);
    }
    FDCHECK(hipGetLastError(), "k_vaskip launch");
  }
  if (layout) {
    if (c->fast->cmode == 1) {
      // a work-list model whose centre has limit rows: its perturbations need the rows'
      // velocity and acceleration terms, so every qvel/qacc perturbation then runs the full
      // pipeline over its own slot (the same layout; results as without skipping). Decided on
      // the device: the gated expansion below turns the flag into the range k_all reads,
      // empty when no centre has rows, so the call needs no host round trip.
      // the perturbations' own inputs, for the full pipeline over them (only when a centre
      // has rows)
      // gated: usually empty, so a few one-wave blocks striding over the range (an empty
      // launch of one 16-wave block per 64 instances took 5 us)
      const long gblk = (ninst - nA + 63)/64;
      hipLaunchKernelGGL(k_fd_expand, dim3((unsigned)(gblk < 256 ? gblk : 256)), dim3(64), 0,
                         c->stream, c->dmodel, c->mirror, B, dq, dv, da,
                         (m.nu ? dc : nullptr), eps, layout, c->fdflag, nA, ninst, 1);
      FDCHECK(hipGetLastError(), "k_fd_expand (fall-back) launch");
      rc = launch_inverse(c, (int)(ninst - nA), nullptr, nullptr, nullptr, nullptr,
                          mjhipSTAGE_NONE, nullptr, 0, skipsensor, c->fdflag + 1);
      if (rc) return rc;
    }
  } else {
    rc = launch_inverse(c, (int)ninst, nullptr, nullptr, nullptr, nullptr, mjhipSTAGE_NONE,
                        nullptr, 0, skipsensor);
    if (rc) return rc;
  }
  if (flg_actuation) {
    hipLaunchKernelGGL(k_fd_act, dim3((ninst + 255)/256), dim3(256), 0, c->stream, c->dmodel,
                       c->mirror, ninst);
    FDCHECK(hipGetLastError(), "k_fd_act launch");
  }
  double *oq = DfDq, *ov = DfDv, *oa = DfDa, *om = DmDq;
  double *sq_ = DsDq, *sv_ = DsDv, *sa_ = DsDa;
  size_t nn = (size_t)B*nv*nv, nm = (size_t)B*nv*m.nM, ns = (size_t)B*nv*m.nsensordata;
  if (!dev) {
    bool ok = true;
    auto dalloc = [&](double* h, size_t n) -> double* {
      if (!h) return nullptr;
      double* d = tmp.alloc(n);
      ok = ok && d;
      return d;
    };
    oq = dalloc(DfDq, nn); ov = dalloc(DfDv, nn); oa = dalloc(DfDa, nn); om = dalloc(DmDq, nm);
    sq_ = dalloc(DsDq, ns); sv_ = dalloc(DsDv, ns); sa_ = dalloc(DsDa, ns);
    if (!ok) {
      set_error("hipMalloc(FD outputs) failed");
      return MJHIP_ERR_HIP;
    }
  }
  long nd = (long)B*(P-1);
  if (oq || ov || oa) {
    hipLaunchKernelGGL(k_fd_dfd, dim3((nd*nv + 255)/256), dim3(256), 0, c->stream, c->dmodel,
                       c->mirror, B, eps, flg_actuation, oq, ov, oa, layout);
  }
  if (sq_ || sv_ || sa_ || om) {
    hipLaunchKernelGGL(k_fd_diff, dim3((nd + 255)/256), dim3(256), 0, c->stream, c->dmodel,
                       c->mirror, B, eps, flg_actuation, nullptr, nullptr, nullptr, sq_, sv_,
                       sa_, om, layout);
  }
  FDCHECK(hipGetLastError(), "k_fd_diff launch");
  if (!dev) {
    auto get = [&](double* h, const double* d, size_t n) {
      return !h || hipMemcpyAsync(h, d, n*8, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
    };
    bool ok = get(DfDq, oq, nn) && get(DfDv, ov, nn) && get(DfDa, oa, nn) && get(DmDq, om, nm) &&
              get(DsDq, sq_, ns) && get(DsDv, sv_, ns) && get(DsDa, sa_, ns);
    int flags[4] = {0, 0, 0, 0};
    if (ok && layout) {
      ok = hipMemcpyAsync(flags, c->fdflag, sizeof(flags), hipMemcpyDeviceToHost,
                          c->stream) == hipSuccess;
    }
    FDCHECK(ok ? hipStreamSynchronize(c->stream) : hipErrorUnknown, "FD output download");
    if (flags[3]) {
      set_error("mjhip_inverseFDBatch: a k_fdall wave's wait for its centre timed out");
      return MJHIP_ERR_HIP;
    }
  }
#undef FDCHECK
  return MJHIP_OK;
}

MJHIP_API int mjhip_inverseFDBatch(mjhipContext* c, int B, const mjtNum* qpos,
                                   const mjtNum* qvel, const mjtNum* qacc, mjtNum eps,
                                   mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa, mjtNum* DsDq,
                                   mjtNum* DsDv, mjtNum* DsDa, mjtNum* DmDq, int flags) {
  return mjhip_inverseFDBatchEx(c, B, qpos, qvel, qacc, nullptr, eps, 0, DfDq, DfDv, DfDa,
                                DsDq, DsDv, DsDa, DmDq, flags);
}

//---------------------------------- single-instance drop-in ---------------------------------
// The reference's single-mjData entry points run as a batch of one on instance 0 of a
// per-model context: the fields a call reads are uploaded from the host mjhipData, one kernel
// runs the stages the reference function runs, and the fields it writes come back.

MJHIP_API int mjhip_modelCapacity(const mjhipModel* m, int* efc_rows, int* contacts) {
  if (!m) return MJHIP_ERR_ARG;
  if (efc_rows) *efc_rows = mjhip_efcCapacity(m);
  if (contacts) *contacts = mjhip_contactCapacity(m, nullptr);
  return MJHIP_OK;
}

// one stage of mj_inverseSkip (or a helper it calls) on instance 0 (the reference function
// is named in the comment); lane 0 of one 64-lane block runs it. ST_INV is the whole
// mj_inverseSkip on the unfused path, which leaves every constraint row in the mirror.
extern "C++" {
enum { ST_INV = 0, ST_POS, ST_VEL, ST_CON, ST_RNE0, ST_RNE1, ST_XFRC };
template <bool CONTACT>
__global__ __launch_bounds__(64) void k_stage(mjhipModel m, Mirror mr, int what, int skipstage,
                                              int skipsensor, int* __restrict__ status) {
  if (threadIdx.x) return;
  Lane<64> d = lane_view(mr, 0, 0);
  int st = 0;
  switch (what) {
    case ST_INV: st = mjh::inverseSkip<64, CONTACT, false>(m, d, skipstage, skipsensor); break;
    case ST_POS: mjh::invPosition<64, CONTACT, false>(m, d, &st); break;   // mj_invPosition
    case ST_VEL: mjh::invVelocity<64, false>(m, d); break;                 // mj_invVelocity
    case ST_CON: mjh::invConstraint(m, d); break;                          // mj_invConstraint
    case ST_RNE0: mjh::rne(m, d, 0, d.qfrc_tmp); break;                    // mj_rne(flg_acc=0)
    case ST_RNE1: mjh::rne(m, d, 1, d.qfrc_tmp); break;                    // mj_rne(flg_acc=1)
    case ST_XFRC: mjh::xfrcAccumulate(m, d, d.qfrc_tmp); break;            // mj_xfrcAccumulate
  }
  if (status) status[0] = st;
}
}  // extern "C++"

static int g_device = 0;
static std::mutex g_mu;
// contexts of the single-instance calls, keyed by the model's content signature (sizes,
// options, every array): a new or edited model at a reused address gets its own context.
// A call leases its entry for its whole upload/launch/download sequence: the lease holds a
// reference (an entry evicted or released meanwhile is freed when its last lease ends) and
// the entry's call lock (the calls share instance 0 and the stream of the context).
struct CtxEntry {
  unsigned long long sig = 0;
  mjhipContext* c = nullptr;
  std::mutex call_mu;
  ~CtxEntry() { if (c) mjhip_contextFree(c); }
};
using CtxRef = std::shared_ptr<CtxEntry>;
// most recently used last, at most kMaxCtx; never destroyed (contexts are not freed during
// static destruction, after the HIP runtime may have gone)
static std::vector<CtxRef>& g_ctx = *new std::vector<CtxRef>;
static const size_t kMaxCtx = 16;
// mjhip_inverseFD's context (capacity 3nv+1) is cached under the signature with this salt
static const unsigned long long kFDSalt = 0x9E3779B97F4A7C15ull;

struct CtxLease {
  CtxRef e;
  std::unique_lock<std::mutex> lk;
  mjhipContext* get() const { return e ? e->c : nullptr; }
};

static CtxLease lease_ctx(const mjhipModel* m, unsigned long long salt, int capacity) {
  const unsigned long long sig = model_signature(m) ^ salt;
  CtxRef e;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (size_t i = 0; i < g_ctx.size(); i++) {
      if (g_ctx[i]->sig == sig) {
        e = g_ctx[i];
        g_ctx.erase(g_ctx.begin() + i);
        g_ctx.push_back(e);
        break;
      }
    }
    if (!e) {
      mjhipContext* c = nullptr;
      if (mjhip_contextCreate(m, g_device, capacity, &c) != MJHIP_OK) return {};
      e = std::make_shared<CtxEntry>();
      e->sig = sig;
      e->c = c;
      if (g_ctx.size() >= kMaxCtx) g_ctx.erase(g_ctx.begin());   // least recently used
      g_ctx.push_back(e);
    }
  }
  CtxLease L;
  L.e = e;
  L.lk = std::unique_lock<std::mutex>(e->call_mu);
  return L;
}

static void report(const char* what) {
  std::string msg = std::string(what) + ": " + g_last_error;
  if (g_error_cb) {
    g_error_cb(msg.c_str());
  } else {
    fprintf(stderr, "mjhip error: %s\n", msg.c_str());
  }
}

MJHIP_API void mjhip_setDevice(int device) { g_device = device; }

MJHIP_API void mjhip_releaseModel(const mjhipModel* m) {
  const unsigned long long sig = model_signature(m);
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t i = g_ctx.size(); i-- > 0;) {
    if (g_ctx[i]->sig == sig || g_ctx[i]->sig == (sig ^ kFDSalt)) g_ctx.erase(g_ctx.begin() + i);
  }
}

extern "C++" {
// instance 0 of a mirror field: element k at F[k*64] (block 0, lane 0), or at F[k] for an
// instance-contiguous field (the XSCC / XSIC fields)
template <class T>
static int put0(mjhipContext* c, T* dev, const T* host, long n) {
  if (n <= 0 || !dev || !host) return MJHIP_OK;
  if (c->contig_ptr.count((const void*)dev)) {
    HIPCHECK(hipMemcpyAsync(dev, host, sizeof(T)*n, hipMemcpyHostToDevice, c->stream));
    return MJHIP_OK;
  }
  HIPCHECK(hipMemcpy2DAsync(dev, 64*sizeof(T), host, sizeof(T), sizeof(T), n,
                            hipMemcpyHostToDevice, c->stream));
  return MJHIP_OK;
}

template <class T>
static int get0(mjhipContext* c, T* host, const T* dev, long n) {
  if (n <= 0 || !dev || !host) return MJHIP_OK;
  if (c->contig_ptr.count((const void*)dev)) {
    HIPCHECK(hipMemcpyAsync(host, dev, sizeof(T)*n, hipMemcpyDeviceToHost, c->stream));
    return MJHIP_OK;
  }
  HIPCHECK(hipMemcpy2DAsync(host, sizeof(T), dev, 64*sizeof(T), sizeof(T), n,
                            hipMemcpyDeviceToHost, c->stream));
  return MJHIP_OK;
}
}  // extern "C++"

// data fields of stages lo..hi (MJHIP_DATA_FIELDS stage numbers) host -> instance 0
static int put_stages(mjhipContext* c, const mjhipModel* m, const mjhipData* d, int lo, int hi) {
  int rc = 0;
#define MJ_M(n) m->n
#define XD(name, d0, d1, stage)                                                          \
  if (!rc && stage >= lo && stage <= hi) rc = put0(c, c->mirror.name, (const double*)d->name, \
                                                   (long)(m->d0) * (d1));
  MJHIP_DATA_FIELDS
#undef XD
#undef MJ_M
  return rc;
}

static int get_stages(mjhipContext* c, const mjhipModel* m, mjhipData* d, int lo, int hi) {
  int rc = 0;
#define MJ_M(n) m->n
#define XD(name, d0, d1, stage)                                                          \
  if (!rc && stage >= lo && stage <= hi) rc = get0(c, d->name, (const double*)c->mirror.name, \
                                                   (long)(m->d0) * (d1));
  MJHIP_DATA_FIELDS
#undef XD
#undef MJ_M
  return rc;
}

// constraint rows (XE) and contacts (XC) written by stages lo..hi, host -> instance 0, with
// the counts. Rows beyond the context's capacity cannot come from a supported model.
static int put_rows(mjhipContext* c, const mjhipModel* m, const mjhipData* d, int lo, int hi) {
  if (d->nefc > c->efc_cap || d->ncon > c->con_cap || d->nefc < 0 || d->ncon < 0) {
    set_error("%d constraint rows / %d contacts exceed the model's device capacity (%d / %d)",
              d->nefc, d->ncon, c->efc_cap, c->con_cap);
    return MJHIP_ERR_CAPACITY;
  }
  if ((d->nefc && d->efc_capacity < d->nefc) || (d->ncon && d->con_capacity < d->ncon)) {
    set_error("mjhipData holds %d rows / %d contacts but capacities %d / %d",
              d->nefc, d->ncon, d->efc_capacity, d->con_capacity);
    return MJHIP_ERR_ARG;
  }
  // sparse-mode models: compressed rows (nJ values) and the tendon rows' structure
  const bool sparse = mjh_isSparse(m);
  if (sparse && lo <= 1 && hi >= 1) {
    if (d->nJ < 0 || d->nJ > c->mirror.nj_cap) {
      set_error("%d compressed Jacobian entries exceed the device capacity (%ld)", d->nJ,
                c->mirror.nj_cap);
      return MJHIP_ERR_CAPACITY;
    }
    if ((m->ntendon && (!d->ten_J_rownnz || !d->ten_J_rowadr || !d->ten_J_colind)) ||
        (d->nefc && (!d->efc_J_rownnz || !d->efc_J_rowadr || !d->efc_J_colind || !d->efc_JT ||
                     !d->efc_JT_rownnz || !d->efc_JT_rowadr || !d->efc_JT_colind))) {
      set_error("sparse-Jacobian model: mjhipData lacks the compressed Jacobian arrays");
      return MJHIP_ERR_ARG;
    }
  }
  const int cnt[4] = {d->nefc, d->ne, d->nf, d->nl};
  int rc = put0(c, c->mirror.efc_count, cnt, 4);
  if (!rc) rc = put0(c, c->mirror.con_count, &d->ncon, 1);
  const int nv = m->nv;
  (void)nv;
#define MJ_M(n) m->n
#define XE(type, name, w, stage) \
  if (!rc && stage >= lo && stage <= hi) \
    rc = put0(c, c->mirror.name, (const type*)d->name, \
              (sparse && !strcmp(#name, "efc_J")) ? (long)d->nJ : (long)d->nefc * (w));
  MJHIP_DATA_EFC
#undef XE
  if (!rc && sparse && lo <= 1 && hi >= 1) {
    const long nt = m->ntendon, nJ = d->nJ, ne = d->nefc;
    rc = put0(c, c->mirror.nJ, &d->nJ, 1);
    if (!rc) rc = put0(c, c->mirror.ten_J_rownnz, (const int*)d->ten_J_rownnz, nt);
    if (!rc) rc = put0(c, c->mirror.ten_J_rowadr, (const int*)d->ten_J_rowadr, nt);
    if (!rc) rc = put0(c, c->mirror.ten_J_colind, (const int*)d->ten_J_colind, nt*nv);
    if (!rc) rc = put0(c, c->mirror.efc_J_rownnz, (const int*)d->efc_J_rownnz, ne);
    if (!rc) rc = put0(c, c->mirror.efc_J_rowadr, (const int*)d->efc_J_rowadr, ne);
    if (!rc) rc = put0(c, c->mirror.efc_J_colind, (const int*)d->efc_J_colind, nJ);
    if (!rc) rc = put0(c, c->mirror.efc_JT, (const double*)d->efc_JT, nJ);
    if (!rc && ne) rc = put0(c, c->mirror.efc_JT_rownnz, (const int*)d->efc_JT_rownnz, (long)nv);
    if (!rc && ne) rc = put0(c, c->mirror.efc_JT_rowadr, (const int*)d->efc_JT_rowadr, (long)nv);
    if (!rc) rc = put0(c, c->mirror.efc_JT_colind, (const int*)d->efc_JT_colind, nJ);
  }
#define XC(type, name, w, stage) \
  if (!rc && stage >= lo && stage <= hi) rc = put0(c, c->mirror.name, (const type*)d->name, \
                                                   (long)d->ncon * (w));
  MJHIP_DATA_CONTACT
#undef XC
#undef MJ_M
  return rc;
}

// rows written by stages lo..hi, instance 0 -> host, and the counts (contacts when lo <= 1);
// the caller synchronizes. Reading the counts needs one blocking copy first.
static int get_rows(mjhipContext* c, const mjhipModel* m, mjhipData* d, int lo, int hi) {
  int cnt[4] = {0, 0, 0, 0}, ncon = 0, nJ = 0;
  const bool sparse = mjh_isSparse(m);
  int rc = get0(c, cnt, (const int*)c->mirror.efc_count, 4);
  if (!rc) rc = get0(c, &ncon, (const int*)c->mirror.con_count, 1);
  if (!rc && sparse) rc = get0(c, &nJ, (const int*)c->mirror.nJ, 1);
  if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) {
    set_error("hipStreamSynchronize failed");
    rc = MJHIP_ERR_HIP;
  }
  if (rc) return rc;
  d->nefc = cnt[0]; d->ne = cnt[1]; d->nf = cnt[2]; d->nl = cnt[3];
  if (lo <= 1) d->ncon = ncon;
  if (sparse && lo <= 1) d->nJ = nJ;
  if (sparse && lo <= 1 &&
      ((m->ntendon && (!d->ten_J_rownnz || !d->ten_J_rowadr || !d->ten_J_colind)) ||
       (cnt[0] && d->efc_capacity >= cnt[0] &&
        (!d->efc_J_rownnz || !d->efc_J_rowadr || !d->efc_J_colind || !d->efc_JT ||
         !d->efc_JT_rownnz || !d->efc_JT_rowadr || !d->efc_JT_colind)))) {
    set_error("sparse-Jacobian model: mjhipData lacks the compressed Jacobian arrays");
    return MJHIP_ERR_ARG;
  }
  // rows a caller's buffers cannot hold: mjWARN_CNSTRFULL analogue, nothing written
  if ((cnt[0] && d->efc_capacity < cnt[0]) || (lo <= 1 && ncon && d->con_capacity < ncon)) {
    if (d->efc_capacity > 0 || d->con_capacity > 0) d->status |= MJHIP_INST_CNSTRFULL;
    return MJHIP_OK;
  }
  const int nv = m->nv;
  (void)nv;
#define MJ_M(n) m->n
#define XE(type, name, w, stage) \
  if (!rc && stage >= lo && stage <= hi) \
    rc = get0(c, (type*)d->name, (const type*)c->mirror.name, \
              (sparse && !strcmp(#name, "efc_J")) ? (long)nJ : (long)cnt[0] * (w));
  MJHIP_DATA_EFC
#undef XE
  if (!rc && sparse && lo <= 1) {
    const long nt = m->ntendon, ne = cnt[0];
    rc = get0(c, (int*)d->ten_J_rownnz, (const int*)c->mirror.ten_J_rownnz, nt);
    if (!rc) rc = get0(c, (int*)d->ten_J_rowadr, (const int*)c->mirror.ten_J_rowadr, nt);
    if (!rc) rc = get0(c, (int*)d->ten_J_colind, (const int*)c->mirror.ten_J_colind, nt*nv);
    if (!rc) rc = get0(c, (int*)d->efc_J_rownnz, (const int*)c->mirror.efc_J_rownnz, ne);
    if (!rc) rc = get0(c, (int*)d->efc_J_rowadr, (const int*)c->mirror.efc_J_rowadr, ne);
    if (!rc) rc = get0(c, (int*)d->efc_J_colind, (const int*)c->mirror.efc_J_colind, (long)nJ);
    if (!rc) rc = get0(c, (double*)d->efc_JT, (const double*)c->mirror.efc_JT, (long)nJ);
    if (!rc && ne) rc = get0(c, (int*)d->efc_JT_rownnz, (const int*)c->mirror.efc_JT_rownnz, (long)nv);
    if (!rc && ne) rc = get0(c, (int*)d->efc_JT_rowadr, (const int*)c->mirror.efc_JT_rowadr, (long)nv);
    if (!rc) rc = get0(c, (int*)d->efc_JT_colind, (const int*)c->mirror.efc_JT_colind, (long)nJ);
  }
#define XC(type, name, w, stage) \
  if (!rc && lo <= 1 && stage >= lo && stage <= hi) \
    rc = get0(c, (type*)d->name, (const type*)c->mirror.name, (long)ncon * (w));
  MJHIP_DATA_CONTACT
#undef XC
#undef MJ_M
  return rc;
}

static int sync_stream(mjhipContext* c) {
  HIPCHECK(hipStreamSynchronize(c->stream));
  return MJHIP_OK;
}

// run one k_stage on instance 0; status comes back into d->status
static int run_stage(mjhipContext* c, mjhipData* d, int what, int skipstage = 0,
                     int skipsensor = 1) {
  if (c->con_cap > 0) {
    hipLaunchKernelGGL(k_stage<true>, dim3(1), dim3(64), 0, c->stream, c->dmodel, c->mirror,
                       what, skipstage, skipsensor, c->status);
  } else {
    hipLaunchKernelGGL(k_stage<false>, dim3(1), dim3(64), 0, c->stream, c->dmodel, c->mirror,
                       what, skipstage, skipsensor, c->status);
  }
  HIPCHECK(hipGetLastError());
  int st = 0;
  if (int rc = get0(c, &st, (const int*)c->status, 1)) return rc;
  if (int rc = sync_stream(c)) return rc;
  d->status = st;
  return MJHIP_OK;
}

// upload the fields a skipped stage reads (data fields, constraint rows, contacts), run one
// instance, download every output field of the stages that ran
MJHIP_API void mjhip_inverseSkip(const mjhipModel* m, mjhipData* d, int skipstage,
                                 int skipsensor) {
  CtxLease lease = lease_ctx(m, 0, 64);
  mjhipContext* c = lease.get();
  if (!c) {
    report("mjhip_inverseSkip");
    return;
  }
  int rc = hipSetDevice(c->device) == hipSuccess ? 0 : MJHIP_ERR_HIP;
  if (!rc) rc = put_stages(c, m, d, 0, skipstage);
  // the constraint rows of the skipped stages: mj_makeConstraint's (skipstage >= POS) and
  // mj_referenceConstraint's efc_vel / efc_aref (skipstage >= VEL)
  if (!rc && skipstage >= mjhipSTAGE_POS) rc = put_rows(c, m, d, 1, skipstage);
  if (!rc && m->nsensor > 0) {
    // sensor inputs: the values of skipped stages' sensors are kept (sensordata), and the
    // mjData inputs some sensors read (clock: time; force/torque/accelerometer via
    // mj_rnePostConstraint: xfrc_applied; actuatorfrc/jointactuatorfrc)
    if (skipstage > mjhipSTAGE_NONE && d->sensordata)
      rc = put0(c, c->mirror.sensordata, (const double*)d->sensordata, m->nsensordata);
    if (!rc) rc = put0(c, c->mirror.time, &d->time, 1);
    if (!rc && d->xfrc_applied) rc = put0(c, c->mirror.xfrc_applied, (const double*)d->xfrc_applied,
                                          6L*m->nbody);
    if (!rc && d->actuator_force) rc = put0(c, c->mirror.actuator_force,
                                            (const double*)d->actuator_force, (long)m->nu);
    if (!rc && d->qfrc_actuator) rc = put0(c, c->mirror.qfrc_actuator,
                                           (const double*)d->qfrc_actuator, (long)m->nv);
  }
  if (!rc && (skipstage < mjhipSTAGE_NONE || skipstage > mjhipSTAGE_VEL)) {
    set_error("skipstage must be mjSTAGE_NONE, mjSTAGE_POS or mjSTAGE_VEL");
    rc = MJHIP_ERR_ARG;
  }
  if (!rc) rc = run_stage(c, d, ST_INV, skipstage, skipsensor);
  if (!rc) rc = get_stages(c, m, d, skipstage + 1, 3);
  if (!rc && m->nsensor > 0 && !skipsensor) {
    // mjData fields the sensor stages computed on demand (scratch sized 0 when unneeded)
#define MJ_M(n) m->n
#define XD(name, d0, d1, stage)                                                     \
    if (!rc && d->name && c->mirror.name##_n > 0)                                    \
      rc = get0(c, d->name, (const double*)c->mirror.name, (long)(m->d0) * (d1));
    MJHIP_DATA_SENSOR_AUX
#undef XD
#undef MJ_M
  }
  mjtNum e[2] = {0, 0};
  const bool energy = (m->opt.enableflags & mjhipENBL_ENERGY) && skipstage < mjhipSTAGE_VEL;
  if (!rc && energy) rc = get0(c, e, (const double*)c->mirror.energy, 2);
  // the rows of the stages that ran (and the counts); get_rows synchronizes the stream
  if (!rc) rc = get_rows(c, m, d, skipstage + 1, 3);
  if (!rc) rc = sync_stream(c);
  if (!rc && energy) {
    // mj_energyPos/Vel write the energy of the stages that ran (engine_inverse.c:207-223)
    if (skipstage < mjhipSTAGE_POS) d->energy[0] = e[0];
    d->energy[1] = e[1];
  }
  if (rc) report("mjhip_inverseSkip");
}

MJHIP_API void mjhip_inverse(const mjhipModel* m, mjhipData* d) {
  mjhip_inverseSkip(m, d, mjhipSTAGE_NONE, 0);
}

// mj_invPosition / mj_invVelocity / mj_invConstraint (engine_inverse.c:37-76, :169-192): only
// that stage runs, it reads the inputs and earlier stages' fields from d and writes only its
// own outputs into d
static void single_stage(const mjhipModel* m, mjhipData* d, int what, const char* name) {
  CtxLease lease = lease_ctx(m, 0, 64);
  mjhipContext* c = lease.get();
  int rc = c ? 0 : MJHIP_ERR_HIP;
  if (!rc && hipSetDevice(c->device) != hipSuccess) rc = MJHIP_ERR_HIP;
  const int stage = what;                  // ST_POS/VEL/CON = position/velocity/acceleration
  if (!rc) rc = put_stages(c, m, d, 0, stage - 1);
  if (!rc && stage > ST_POS) rc = put_rows(c, m, d, 1, stage - 1);
  if (!rc) rc = run_stage(c, d, what);
  if (!rc) {
    if (what == ST_CON) {                  // qfrc_constraint only (qfrc_inverse is not its output)
      rc = get0(c, d->qfrc_constraint, (const double*)c->mirror.qfrc_constraint, (long)m->nv);
    } else {
      rc = get_stages(c, m, d, stage, stage);
    }
  }
  if (!rc) rc = get_rows(c, m, d, stage, stage);
  if (!rc) rc = sync_stream(c);
  if (rc) report(name);
}

MJHIP_API void mjhip_invPosition(const mjhipModel* m, mjhipData* d) {
  single_stage(m, d, ST_POS, "mjhip_invPosition");
}

MJHIP_API void mjhip_invVelocity(const mjhipModel* m, mjhipData* d) {
  single_stage(m, d, ST_VEL, "mjhip_invVelocity");
}

MJHIP_API void mjhip_invConstraint(const mjhipModel* m, mjhipData* d) {
  single_stage(m, d, ST_CON, "mjhip_invConstraint");
}

// mj_rne (engine_core_smooth.c:1969-2023): reads the caller's cdof, cinert, cvel, cdof_dot,
// qvel (and qacc with flg_acc) and writes only `result`
MJHIP_API void mjhip_rne(const mjhipModel* m, mjhipData* d, int flg_acc, mjtNum* result) {
  CtxLease lease = lease_ctx(m, 0, 64);
  mjhipContext* c = lease.get();
  int rc = c ? 0 : MJHIP_ERR_HIP;
  if (!rc && hipSetDevice(c->device) != hipSuccess) rc = MJHIP_ERR_HIP;
  if (!rc) rc = put0(c, c->mirror.cdof, (const double*)d->cdof, 6L*m->nv);
  if (!rc) rc = put0(c, c->mirror.cinert, (const double*)d->cinert, 10L*m->nbody);
  if (!rc) rc = put0(c, c->mirror.cvel, (const double*)d->cvel, 6L*m->nbody);
  if (!rc) rc = put0(c, c->mirror.cdof_dot, (const double*)d->cdof_dot, 6L*m->nv);
  if (!rc) rc = put0(c, c->mirror.qvel, (const double*)d->qvel, (long)m->nv);
  if (!rc && flg_acc) rc = put0(c, c->mirror.qacc, (const double*)d->qacc, (long)m->nv);
  int st = d->status;
  if (!rc) rc = run_stage(c, d, flg_acc ? ST_RNE1 : ST_RNE0);
  d->status = st;                          // mj_rne leaves d alone
  if (!rc && result) rc = get0(c, result, (const double*)c->mirror.qfrc_tmp, (long)m->nv);
  if (!rc) rc = sync_stream(c);
  if (rc) report("mjhip_rne");
}

// mj_xfrcAccumulate (engine_support.c:1254-1261): qfrc += J' xfrc_applied over bodies 1..,
// through mj_applyFT (its mj_jac reads d's xipos, subtree_com and cdof)
MJHIP_API void mjhip_xfrcAccumulate(const mjhipModel* m, mjhipData* d, mjtNum* qfrc) {
  CtxLease lease = lease_ctx(m, 0, 64);
  mjhipContext* c = lease.get();
  int rc = c ? 0 : MJHIP_ERR_HIP;
  if (!rc && hipSetDevice(c->device) != hipSuccess) rc = MJHIP_ERR_HIP;
  if (!rc) rc = put0(c, c->mirror.xipos, (const double*)d->xipos, 3L*m->nbody);
  if (!rc) rc = put0(c, c->mirror.subtree_com, (const double*)d->subtree_com, 3L*m->nbody);
  if (!rc) rc = put0(c, c->mirror.cdof, (const double*)d->cdof, 6L*m->nv);
  if (!rc) rc = put0(c, c->mirror.xfrc_applied, (const double*)d->xfrc_applied, 6L*m->nbody);
  if (!rc) rc = put0(c, c->mirror.qfrc_tmp, (const double*)qfrc, (long)m->nv);
  int st = d->status;
  if (!rc) rc = run_stage(c, d, ST_XFRC);
  d->status = st;
  if (!rc) rc = get0(c, qfrc, (const double*)c->mirror.qfrc_tmp, (long)m->nv);
  if (!rc) rc = sync_stream(c);
  if (rc) report("mjhip_xfrcAccumulate");
}

// mju_dot (engine_util_blas.c:680-741, four partial sums) and mju_norm, for the two norms of
// mj_compareFwdInv
static double dot4(const double* a, const double* b, int n) {
  double r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    r0 += a[i]*b[i];
    r1 += a[i+1]*b[i+1];
    r2 += a[i+2]*b[i+2];
    r3 += a[i+3]*b[i+3];
  }
  double res = (r0 + r2) + (r1 + r3);
  const int left = n - i;           // the tail is one sum added to res, as mju_dot's
  if (left == 3) {
    res += a[i]*b[i] + a[i+1]*b[i+1] + a[i+2]*b[i+2];
  } else if (left == 2) {
    res += a[i]*b[i] + a[i+1]*b[i+1];
  } else if (left == 1) {
    res += a[i]*b[i];
  }
  return res;
}

// mj_compareFwdInv (engine_inverse.c:275-316): with constraint rows, qforce = qfrc_applied +
// qfrc_actuator + J'xfrc_applied (mj_xfrcAccumulate) is what inverse dynamics of the forward
// pass's qacc must return; mj_inverseSkip(VEL, 1) runs on the device with the forward pass's
// rows; solver_fwdinv = (|fwd - inv qfrc_constraint|, |qforce - qfrc_inverse|); the forward
// qfrc_constraint and efc_force are restored.
MJHIP_API void mjhip_compareFwdInv(const mjhipModel* m, mjhipData* d) {
  const int nv = m->nv, nefc = d->nefc;
  d->solver_fwdinv[0] = d->solver_fwdinv[1] = 0;
  if (!nefc) return;
  if (!d->efc_force || d->efc_capacity < nefc) {
    set_error("mj_compareFwdInv: the data holds no constraint rows (efc_capacity %d < nefc %d)",
              d->efc_capacity, nefc);
    report("mjhip_compareFwdInv");
    return;
  }
  std::vector<double> qforce(nv), dif(nv), save_qc(d->qfrc_constraint, d->qfrc_constraint + nv),
                      save_force(d->efc_force, d->efc_force + nefc);
  for (int i = 0; i < nv; i++) qforce[i] = d->qfrc_applied[i] + d->qfrc_actuator[i];
  mjhip_xfrcAccumulate(m, d, qforce.data());
  mjhip_inverseSkip(m, d, mjhipSTAGE_VEL, 1);
  for (int i = 0; i < nv; i++) dif[i] = save_qc[i] - d->qfrc_constraint[i];
  d->solver_fwdinv[0] = sqrt(dot4(dif.data(), dif.data(), nv));
  for (int i = 0; i < nv; i++) dif[i] = qforce[i] - d->qfrc_inverse[i];
  d->solver_fwdinv[1] = sqrt(dot4(dif.data(), dif.data(), nv));
  memcpy(d->qfrc_constraint, save_qc.data(), sizeof(double)*nv);
  memcpy(d->efc_force, save_force.data(), sizeof(double)*nefc);
}

// mjd_inverseFD (engine_derivative_fd.c:611-719, mujoco.h:1244-1247) for one mjData: the
// batched FD with one base state (d's qpos, qvel, qacc, ctrl). Like the reference, d is left
// with the outputs of the last evaluation (the last qpos perturbation) and its own qpos.
MJHIP_API void mjhip_inverseFD(const mjhipModel* m, mjhipData* d, mjtNum eps,
                               mjtByte flg_actuation, mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa,
                               mjtNum* DsDq, mjtNum* DsDv, mjtNum* DsDa, mjtNum* DmDq) {
  const int P = 3*m->nv + 1;
  // an FD batch of one needs 3nv+1 instances: a context of that capacity, leased like the
  // single-instance ones under the salted signature
  CtxLease lease = lease_ctx(m, kFDSalt, P);
  mjhipContext* c = lease.get();
  int rc = c ? 0 : MJHIP_ERR_HIP;
  if (!rc && m->nsensor && (DsDq || DsDv || DsDa)) {
    std::vector<double> t(P, d->time);                    // clock sensors of every evaluation
    rc = mjhip_mirrorUpload(c, "time", 0, P, t.data());
  }
  if (!rc) rc = mjhip_inverseFDBatchEx(c, 1, d->qpos, d->qvel, d->qacc, d->ctrl, eps,
                                       flg_actuation, DfDq, DfDv, DfDa, DsDq, DsDv, DsDa, DmDq,
                                       kFlagFDFull);
  if (!rc) {
    // the reference's last evaluation (engine_derivative_fd.c:646-715): the last qpos
    // perturbation, else the last qvel one, else the last qacc one, else the centre
    const int nv = m->nv;
    const int last = (DfDq || DsDq || DmDq) ? P - 1 : (DfDv || DsDv) ? 2*nv
                     : (DfDa || DsDa) ? nv : 0;
    std::vector<double> keep(d->qpos, d->qpos + m->nq);
#define MJ_M(n) m->n
#define XD(name, d0, d1, stage)                                                     \
    if (!rc && d->name && stage > 0 && (m->d0) * (d1) > 0)                           \
      rc = mjhip_mirrorDownload(c, #name, last, 1, d->name);
    MJHIP_DATA_FIELDS
#undef XD
#undef MJ_M
    memcpy(d->qpos, keep.data(), sizeof(double)*m->nq);
  }
  if (rc) report("mjhip_inverseFD");
}

}  // extern "C"
