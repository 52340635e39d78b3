// engine_device.h — per-instance mj_inverseSkip pipeline for the HIP engine.
//
// One lane = one simulation instance. Every per-instance array lives in the device mirror
// (include/mjhip.h: F[(blk*S + k)*64 + lane]); `Lane<STRIDE>` is a strided view of one
// lane's slice, so the code below indexes fields exactly like the reference indexes mjData
// (e.g. d.xmat[9*i+k]) while every access of a wavefront is one contiguous 512-byte segment.
// STRIDE = 64 on the GPU; the test suite also compiles this file for the host with
// STRIDE = 1 (tests/cpu_kernel_harness.cpp) to check it bit-for-bit against the oracle.
//
// Each function cites the reference file:line it restates (paths relative to the
// reference root). Summation orders follow the reference's scalar C code.
#ifndef MJHIP_ENGINE_DEVICE_H_
#define MJHIP_ENGINE_DEVICE_H_

#include <math.h>

#include "../../include/mjhip.h"
#include "../../include/mjhip_contact.h"

#if defined(__HIPCC__)
  #define MJH_LAMBDA_INLINE __attribute__((always_inline))
#else
  #define MJH_LAMBDA_INLINE
#endif
#if defined(__HIPCC__)
  // always inlined: an out-of-line call would pass the Lane view and the model through
  // private (scratch) memory and reload every field pointer from there
  #define MJH_HD __host__ __device__ inline __attribute__((always_inline))
#else
  #define MJH_HD inline
#endif

// Per-stage timers (mjhip_contextTimers: the reference's mjTIMER_* table, include/mjhip.h).
// While a context has them on, mjh_tbuf points at its accumulator (MJH_TSLOTS counters) and
// lane 0 of every wave adds the 100 MHz wall clock at each phase mark, so the mean over
// waves of mark k minus mark k-1 is the mean wall time a wave spends in phase k; a group's
// first mark also counts the waves. Null otherwise: one scalar load and a branch per mark.
// Marks: generic k_inverse 0-9 (waves counted in 24), k_constraint 10-13 (25),
// k_constraint_coop 14-18 (26), the straight-line k_all 19-22 (27). Experiment builds
// (-DMJH_PHASE_TIMING, tools/exp_phases.py) add per-contact spans in slots 40-45.
#define MJH_TSLOTS 48
#if defined(__HIPCC__)
#if defined(MJH_TBUF_EXTERN)                // a run-time code object: found by name
extern "C" {
__device__ unsigned long long* mjh_tbuf = nullptr;
}
#else
static __device__ unsigned long long* mjh_tbuf = nullptr;
#endif
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define MJH_PHASE(k)                                                                  \
  do {                                                                                \
    unsigned long long* tb_ = mjh_tbuf;                                               \
    if (tb_ && (threadIdx.x & 63) == 0) atomicAdd(&tb_[k], wall_clock64());            \
  } while (0)
#define MJH_PHASE0(k, c)                                                              \
  do {                                                                                \
    unsigned long long* tb_ = mjh_tbuf;                                               \
    if (tb_ && (threadIdx.x & 63) == 0) {                                             \
      atomicAdd(&tb_[k], wall_clock64());                                             \
      atomicAdd(&tb_[c], 1ull);                                                       \
    }                                                                                 \
  } while (0)
#else
#define MJH_PHASE(k) do {} while (0)
#define MJH_PHASE0(k, c) do {} while (0)
#endif
#if defined(MJH_PHASE_TIMING) && defined(__HIP_DEVICE_COMPILE__)
// spans inside a lane's own work (lane 0's): MJH_TICK(t) reads the clock, MJH_SPAN(k, a, b)
// adds b - a to slot 40 + k (slot 41 + k counts the spans)
#define MJH_TICK(t) const unsigned long long t = wall_clock64()
#define MJH_SPAN(k, a, b)                                                             \
  do {                                                                                \
    unsigned long long* tb_ = mjh_tbuf;                                               \
    if (tb_ && (threadIdx.x & 63) == 0) {                                             \
      atomicAdd(&tb_[40 + (k)], (b) - (a));                                           \
      atomicAdd(&tb_[41 + (k)], 1ull);                                                \
    }                                                                                 \
  } while (0)
#else
#define MJH_TICK(t) do {} while (0)
#define MJH_SPAN(k, a, b) do {} while (0)
#endif

// a streaming (non-temporal) store of a mirror value the kernel does not read back (the
// generated kernels, codegen.NT_STORES); a plain store in host builds and with -DMJHIP_NO_NT
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MJHIP_NO_NT)
#define MJH_NT_STORE(lv, v) __builtin_nontemporal_store((double)(v), &(lv))
#define MJH_NT_LOAD(lv) __builtin_nontemporal_load(&(lv))
#else
#define MJH_NT_STORE(lv, v) ((lv) = (v))
#define MJH_NT_LOAD(lv) (lv)
#endif
// a load that streams in one instantiation of a generated kernel (nt a template argument)
#define MJH_NT_LOAD_IF(nt, lv) ((nt) ? MJH_NT_LOAD(lv) : (lv))
// a store that streams in one instantiation of a generated kernel (nt a template argument)
#define MJH_NT_STORE_IF(nt, lv, v)                                                      \
  do {                                                                                  \
    if constexpr (nt) { MJH_NT_STORE(lv, v); } else { (lv) = (v); }                     \
  } while (0)

// mjtSensor values (include/mujoco/mjmodel.h)
enum { mjhSENS_TOUCH = 0, mjhSENS_ACCELEROMETER, mjhSENS_VELOCIMETER, mjhSENS_GYRO,
       mjhSENS_FORCE, mjhSENS_TORQUE, mjhSENS_MAGNETOMETER, mjhSENS_RANGEFINDER,
       mjhSENS_CAMPROJECTION, mjhSENS_JOINTPOS, mjhSENS_JOINTVEL, mjhSENS_TENDONPOS,
       mjhSENS_TENDONVEL, mjhSENS_ACTUATORPOS, mjhSENS_ACTUATORVEL, mjhSENS_ACTUATORFRC,
       mjhSENS_JOINTACTFRC, mjhSENS_BALLQUAT, mjhSENS_BALLANGVEL, mjhSENS_JOINTLIMITPOS,
       mjhSENS_JOINTLIMITVEL, mjhSENS_JOINTLIMITFRC, mjhSENS_TENDONLIMITPOS,
       mjhSENS_TENDONLIMITVEL, mjhSENS_TENDONLIMITFRC, mjhSENS_FRAMEPOS, mjhSENS_FRAMEQUAT,
       mjhSENS_FRAMEXAXIS, mjhSENS_FRAMEYAXIS, mjhSENS_FRAMEZAXIS, mjhSENS_FRAMELINVEL,
       mjhSENS_FRAMEANGVEL, mjhSENS_FRAMELINACC, mjhSENS_FRAMEANGACC, mjhSENS_SUBTREECOM,
       mjhSENS_SUBTREELINVEL, mjhSENS_SUBTREEANGMOM, mjhSENS_GEOMDIST, mjhSENS_GEOMNORMAL,
       mjhSENS_GEOMFROMTO, mjhSENS_E_POTENTIAL, mjhSENS_E_KINETIC, mjhSENS_CLOCK };

// 1 when some sensor needs mj_subtreeVel (engine_sensor.c:552-561) / mj_rnePostConstraint
// (:712-723): their mjData outputs are then allocated as scratch
MJH_HD int mjh_needSubtreeVel(const mjhipModel* m) {
  for (int i = 0; i < m->nsensor; i++) {
    const int t = m->sensor_type[i];
    if (t == mjhSENS_SUBTREELINVEL || t == mjhSENS_SUBTREEANGMOM) return 1;
  }
  return 0;
}
// 1 when a tendon is spatial (two 3 x nv site Jacobians per path segment)
MJH_HD int mjh_needSpatial(const mjhipModel* m) {
  for (int i = 0; i < m->nwrap; i++) {
    if (m->wrap_type[i] != mjhipWRAP_JOINT) return 1;
  }
  return 0;
}
// 1 when an actuator has a slider-crank transmission or a site transmission with a
// reference site (three or four 3 x nv Jacobians at once)
MJH_HD int mjh_needSliderCrank(const mjhipModel* m) {
  for (int i = 0; i < m->nu; i++) {
    if (m->actuator_trntype[i] == mjhipTRN_SLIDERCRANK) return 1;
    if (m->actuator_trntype[i] == mjhipTRN_SITE && m->actuator_trnid[2*i+1] >= 0) return 1;
    if (m->actuator_trntype[i] == mjhipTRN_BODY) return 1;
  }
  return 0;
}
// 1 when a candidate geom pair of the model runs the native GJK/EPA solver (mjc_Convex,
// mjc_ConvexHField): its
// per-instance scratch (mjh::CcdMem) is allocated, 6 ccd_iterations + 6 faces
// mj_isSparse (engine_core_constraint.c:99-106): jacobian="sparse", or "auto" with nv >= 60.
// Such models keep the reference's compressed rows: ten_J (mj_tendon, engine_core_smooth.c:
// 651-860) and efc_J (mj_addConstraint :265-356) hold each row's values over its dof chain,
// with rownnz/rowadr/colind per instance, efc_JT is their transpose (:2083-2104), and J*v and
// J'*f are mju_mulMatVecSparse over the rows of J and JT (:361-377, :426-442). They run the
// generic kernel only (never the fused or cooperative row paths, nor the straight-line kernels).
MJH_HD int mjh_isSparse(const mjhipModel* m) {
  return m->opt.jacobian == mjhipJAC_SPARSE || (m->opt.jacobian == mjhipJAC_AUTO && m->nv >= 60);
}

// dofs of body b and its ancestors (the length of mj_bodyChain, engine_support.c:341-381)
MJH_HD int mjh_chainLength(const mjhipModel* m, int b) {
  int n = 0;
  for (; b > 0; b = m->body_parentid[b]) n += m->body_dofnum[b];
  return n;
}

// an upper bound on the nonzeros of one compressed row of a sparse-mode model: a contact or
// connect/weld row spans two bodies' chains, a tendon row its path's chains (two tendons for a
// tendon coupling), a ball-joint limit 3 dofs (host only: sizes the per-instance CSR arrays)
MJH_HD int mjh_rowNnzMax(const mjhipModel* m) {
  int chain = 0, ten = 0;
  for (int b = 1; b < m->nbody; b++) {
    const int c = mjh_chainLength(m, b);
    chain = c > chain ? c : chain;
  }
  for (int i = 0; i < m->ntendon; i++) {
    int t = 0;
    for (int w = m->tendon_adr[i]; w < m->tendon_adr[i] + m->tendon_num[i]; w++) {
      const int type = m->wrap_type[w], obj = m->wrap_objid[w];
      if (type == mjhipWRAP_JOINT) t += 1;
      else if (type == mjhipWRAP_SITE) t += mjh_chainLength(m, m->site_bodyid[obj]);
      else if (type == mjhipWRAP_SPHERE || type == mjhipWRAP_CYLINDER)
        t += mjh_chainLength(m, m->geom_bodyid[obj]);
    }
    ten = t > ten ? t : ten;
  }
  int r = 2*chain;
  r = 2*ten > r ? 2*ten : r;
  r = r < 3 ? 3 : r;
  return r < m->nv ? r : m->nv;
}

// compressed-row capacity (values) of one instance: efc_cap rows of at most mjh_rowNnzMax
MJH_HD long mjh_njCap(const mjhipModel* m, int efc_cap) {
  return mjh_isSparse(m) ? (long)efc_cap * mjh_rowNnzMax(m) : 0;
}

MJH_HD int mjh_needConvex(const mjhipModel* m) {
  if (!mjhip_contactsEnabled(m)) return 0;
  for (int b1 = 0; b1 < m->nbody; b1++) {
    for (int b2 = b1 + 1; b2 < m->nbody; b2++) {
      if (!mjhip_bodyPairCandidate(m, b1, b2)) continue;
      for (int i = 0; i < m->body_geomnum[b1]; i++) {
        for (int j = 0; j < m->body_geomnum[b2]; j++) {
          int g1 = m->body_geomadr[b1] + i, g2 = m->body_geomadr[b2] + j;
          if (m->geom_type[g1] > m->geom_type[g2]) { int t = g1; g1 = g2; g2 = t; }
          const int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
          if (mjhip_pairUsesCcd(t1, t2) && mjhip_pairMaxContacts(m, t1, t2) > 0 &&
              !mjhip_filterBitmask(m->geom_contype[g1], m->geom_conaffinity[g1],
                                   m->geom_contype[g2], m->geom_conaffinity[g2])) {
            return 1;
          }
        }
      }
    }
  }
  for (int k = 0; k < m->npair; k++) {       // predefined pairs: no bitmask filter
    int t1 = m->geom_type[m->pair_geom1[k]], t2 = m->geom_type[m->pair_geom2[k]];
    if (t1 > t2) { int t = t1; t1 = t2; t2 = t; }
    if (mjhip_pairUsesCcd(t1, t2) && mjhip_pairMaxContacts(m, t1, t2) > 0) return 1;
  }
  return 0;
}
// a geom-distance sensor (mj_geomDistance) whose geom pairs include one the native solver
// measures (mjc_Convex or box-box pairs)
MJH_HD int mjh_needDistanceCcd(const mjhipModel* m) {
  if (m->opt.disableflags & mjhipDSBL_NATIVECCD) return 0;
  for (int i = 0; i < m->nsensor; i++) {
    const int t = m->sensor_type[i];
    if (t < mjhSENS_GEOMDIST || t > mjhSENS_GEOMFROMTO) continue;
    const int o = m->sensor_objid[i], r = m->sensor_refid[i];
    const int n1 = m->sensor_objtype[i] == 1 ? m->body_geomnum[o] : 1;
    const int a1 = m->sensor_objtype[i] == 1 ? m->body_geomadr[o] : o;
    const int n2 = m->sensor_reftype[i] == 1 ? m->body_geomnum[r] : 1;
    const int a2 = m->sensor_reftype[i] == 1 ? m->body_geomadr[r] : r;
    for (int g1 = a1; g1 < a1 + n1; g1++) {
      for (int g2 = a2; g2 < a2 + n2; g2++) {
        int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
        if (t1 > t2) { const int x = t1; t1 = t2; t2 = x; }
        if (mjhip_isConvexPair(t1, t2) || (t1 == mjhipGEOM_BOX && t2 == mjhipGEOM_BOX)) return 1;
      }
    }
  }
  return 0;
}
MJH_HD int mjh_ccdFaceCap(const mjhipModel* m) { return 6*m->opt.ccd_iterations + 6; }
MJH_HD int mjh_needCcd(const mjhipModel* m) {
  return mjh_needConvex(m) || mjh_needDistanceCcd(m);
}
MJH_HD int mjh_ccdDoubles(const mjhipModel* m) {
  return mjh_needCcd(m) ? 72 + 9*(5 + m->opt.ccd_iterations) + 5*mjh_ccdFaceCap(m) : 0;
}
MJH_HD int mjh_ccdInts(const mjhipModel* m) {
  return mjh_needCcd(m) ? 13*mjh_ccdFaceCap(m) : 0;
}
// transmissions the generated kernels leave to the pass after the constraint kernel
// (mjh::transmissionAfter): slider-crank, site and body (adhesion) ones
MJH_HD int mjh_trnAfter(int trn) {
  return trn == mjhipTRN_SLIDERCRANK || trn == mjhipTRN_SITE || trn == mjhipTRN_BODY;
}
MJH_HD int mjh_needTrnAfter(const mjhipModel* m) {
  for (int i = 0; i < m->nu; i++) {
    if (mjh_trnAfter(m->actuator_trntype[i])) return 1;
  }
  return 0;
}
MJH_HD int mjh_needRnePost(const mjhipModel* m) {
  for (int i = 0; i < m->nsensor; i++) {
    const int t = m->sensor_type[i];
    if (t == mjhSENS_ACCELEROMETER || t == mjhSENS_FORCE || t == mjhSENS_TORQUE ||
        t == mjhSENS_FRAMELINACC || t == mjhSENS_FRAMEANGACC) return 1;
  }
  return 0;
}

// 1 when mj_discreteAcc runs the implicit integrator (its mjd_rne_vel scratch is allocated)
MJH_HD int mjh_implicit(const mjhipModel* m) {
  return (m->opt.enableflags & mjhipENBL_INVDISCRETE) && m->opt.integrator == mjhipINT_IMPLICIT;
}

// 1 when mj_discreteAcc's qDeriv has fluid terms (mjd_passive_vel engine_derivative.c:1494-1513
// under the implicit or implicitfast integrator): qDeriv is then held on the D sparsity, and
// Dtmp holds the local 6 x nv Jacobian of each fluid body or geom
MJH_HD int mjh_fluidDeriv(const mjhipModel* m) {
  return (m->opt.enableflags & mjhipENBL_INVDISCRETE) &&
         (m->opt.integrator == mjhipINT_IMPLICIT || m->opt.integrator == mjhipINT_IMPLICITFAST) &&
         !(m->opt.disableflags & mjhipDSBL_PASSIVE) &&
         (m->opt.viscosity > 0 || m->opt.density > 0);
}
MJH_HD int mjh_qDerivStored(const mjhipModel* m) { return mjh_implicit(m) || mjh_fluidDeriv(m); }

// one entry of the static collision program (host-built by coop_program in the order of
// collision_pairs, csrc/pair_program.h), read by the cooperative kernel and collision(): the type-ordered geoms and their types, the pair's contact bound
// (mjhip_pairMaxContacts; < 0: no collision function built here), its margin, and which
// mj_filterSphere test applies with its bound formed as the reference forms it
// (engine_collision_driver.c:1470-1497): filt 0 = bounding spheres, rb1 + rb2 + margin;
// 1 = plane g1, margin + rb2; 2 = plane g2, margin + rb1; 3 = none
struct CoopPair {
  int g1, g2, t1, t2, kmax, filt;
  int b1, b2, rt1, rt2;                     // the geoms' bodies and their roots
  double margin, bound;
};
constexpr int kCoopPairDoubles = (int)(sizeof(CoopPair) / sizeof(double));
static_assert(sizeof(CoopPair) % sizeof(double) == 0, "CoopPair packs into doubles");

namespace mjh {

constexpr double MINVAL = mjhipMINVAL;

// constraint types/states (include/mujoco/mjmodel.h mjtConstraint, mjtConstraintState)
enum { CNSTR_EQUALITY = 0, CNSTR_FRICTION_DOF, CNSTR_FRICTION_TENDON, CNSTR_LIMIT_JOINT,
       CNSTR_LIMIT_TENDON, CNSTR_CONTACT_FRICTIONLESS, CNSTR_CONTACT_PYRAMIDAL,
       CNSTR_CONTACT_ELLIPTIC };
enum { CNSTRSTATE_SATISFIED = 0, CNSTRSTATE_QUADRATIC, CNSTRSTATE_LINEARNEG,
       CNSTRSTATE_LINEARPOS, CNSTRSTATE_CONE };

//---------------------------------- strided per-lane views -----------------------------------

template <int S, class T = double>
struct SP {
  T* p;
  MJH_HD T& operator[](long k) const { return p[k * S]; }
  MJH_HD SP operator+(long k) const { return SP{p + k * S}; }
};

// scratch fields (not part of the mjData contract) and constraint rows (the reference's
// efc_* arena arrays, mjxmacro.h MJDATA_ARENA_POINTERS_SOLVER), per instance.
// XSCC / XSIC mark the instance-contiguous ones: the Jacobian values and column indices,
// whose element a lane touches next depends on its own rows (rowadr, nonzeros), so lanes at
// the same step of a loop address unrelated elements. They keep the block storage of the
// others (64 instances' copies in one block of 64 n elements) but store each instance's n
// elements consecutively, F[(blk*64 + lane)*n + k], so a lane walks its own cache lines
// instead of taking 8 bytes of a line shared with 15 instances that are elsewhere in their
// rows. Where a list is expanded without a definition of its own they read as XSC / XSI.
#define XSCC(name, n) XSC(name, n)
#define XSIC(name, n) XSI(name, n)
#define MJHIP_SCRATCH_FIELDS          \
  XSC(mass_subtree, nbody)            \
  XSC(cacc, 6*nbody)                  \
  XSC(cfrc, 6*nbody)                  \
  XSC(jacp, 3*nv)                     \
  XSC(jacr, 3*nv)                     \
  XSC(jacsc, mjh_needSliderCrank(m)*6*nv) /* slider-crank site Jacobians */ \
  XSC(jact, mjh_needSpatial(m)*6*nv)  /* spatial tendon segment end Jacobians */ \
  XSC(qforce, nv)                     \
  XSC(qfrc_tmp, nv)                   /* single-instance mj_rne / mj_xfrcAccumulate result */ \
  XSC(qacc_save, nv)                  \
  XSC(energy, 2)                      /* mjData energy (mjENBL_ENERGY) */ \
  XSC(time, (m->nsensor > 0))         /* mjData time (clock sensors) */ \
  XSC(subtree_linvel, mjh_needSubtreeVel(m)*3*m->nbody) \
  XSC(subtree_angmom, mjh_needSubtreeVel(m)*3*m->nbody) \
  XSC(body_vel, mjh_needSubtreeVel(m)*6*m->nbody)       \
  XSC(cfrc_int, mjh_needRnePost(m)*6*m->nbody)          \
  XSC(cfrc_ext, mjh_needRnePost(m)*6*m->nbody)          \
  XSC(qDeriv, mjh_qDerivStored(m)*m->nD)  \
  XSC(qLU, mjh_implicit(m)*m->nD)     \
  XSC(Dcvel, mjh_implicit(m)*6*m->nB) \
  XSC(Dcacc, mjh_implicit(m)*6*m->nB) \
  XSC(Dcfrc, mjh_implicit(m)*6*m->nB) \
  XSC(Dcdofdot, mjh_implicit(m)*6*m->nD) \
  XSC(Dtmp, mjh_qDerivStored(m)*6*nv) \
  XSCC(efc_J, mjh_isSparse(m) ? mjh_njCap(m, efc_cap) : (long)efc_cap*nv) \
  XSCC(efc_JT, mjh_njCap(m, efc_cap))   /* sparse mode: the rows' transpose */ \
  XSC(sparse_buf, mjh_isSparse(m)*nv)  /* sparse mode: mju_combineSparse's buffer */ \
  XSCC(efc_pos, efc_cap)               \
  XSCC(efc_margin, efc_cap)            \
  XSCC(efc_frictionloss, efc_cap)      \
  XSCC(efc_diagApprox, efc_cap)        \
  XSCC(efc_KBIP, 4*efc_cap)            \
  XSCC(efc_D, efc_cap)                 \
  XSCC(efc_R, efc_cap)                 \
  XSCC(efc_vel, efc_cap)               \
  XSCC(efc_aref, efc_cap)              \
  XSCC(efc_force, efc_cap)             \
  XSCC(jar, efc_cap)                   \
  XSCC(con_dist, con_cap)              \
  XSCC(con_pos, 3*con_cap)             \
  XSCC(con_frame, 9*con_cap)           \
  XSCC(con_includemargin, con_cap)     \
  XSCC(con_friction, 5*con_cap)        \
  XSCC(con_solref, 2*con_cap)          \
  XSCC(con_solreffriction, 2*con_cap)  \
  XSCC(con_solimp, 5*con_cap)          \
  XSCC(con_mu, con_cap)                \
  XSC(ccd, mjh_ccdDoubles(m))         /* native convex solver (mjh::CcdMem) */

#define MJHIP_SCRATCH_INT_FIELDS      \
  XSIC(efc_type, efc_cap)              \
  XSIC(efc_id, efc_cap)                \
  XSIC(efc_state, efc_cap)             \
  XSIC(efc_J_rownnz, mjh_isSparse(m)*efc_cap)   /* sparse mode: compressed rows */ \
  XSIC(efc_J_rowadr, mjh_isSparse(m)*efc_cap)   \
  XSIC(efc_J_colind, mjh_njCap(m, efc_cap))      \
  XSI(efc_JT_rownnz, mjh_isSparse(m)*nv)         \
  XSI(efc_JT_rowadr, mjh_isSparse(m)*nv)         \
  XSIC(efc_JT_colind, mjh_njCap(m, efc_cap))     \
  XSI(ten_J_rownnz, mjh_isSparse(m)*m->ntendon) \
  XSI(ten_J_rowadr, mjh_isSparse(m)*m->ntendon) \
  XSI(ten_J_colind, mjh_isSparse(m)*m->ntendon*nv) \
  XSI(chainbuf, mjh_isSparse(m)*3*nv)  /* sparse mode: two chains and a merge buffer */ \
  XSI(nJ, mjh_isSparse(m))            /* sparse mode: nonzeros of efc_J */ \
  XSI(efc_count, 4)                   /* nefc, ne, nf, nl */ \
  XSI(con_count, 1)                   /* ncon */ \
  XSIC(con_dim, con_cap)               \
  XSIC(con_geom, 2*con_cap)            \
  XSIC(con_exclude, con_cap)           \
  XSIC(con_efc_address, con_cap)       \
  XSI(ccdi, mjh_ccdInts(m))

template <int S>
struct Lane {
#define XD(name, d0, d1, stage) SP<S> name;
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
#undef XD
#undef XSCC
#undef XSIC
#define XSC(name, n) SP<S> name;
#define XSCC(name, n) SP<1> name;            // instance-contiguous (see the field lists)
  MJHIP_SCRATCH_FIELDS
#undef XSC
#undef XSCC
#define XSI(name, n) SP<S, int> name;
#define XSIC(name, n) SP<1, int> name;
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
#undef XSIC
#define XSCC(name, n) XSC(name, n)
#define XSIC(name, n) XSI(name, n)
  int efc_cap;
  int con_cap;
  long nj_cap;                               // sparse mode: compressed-row capacity (values)
  // fused constraint path only (nbody <= 64): chain[k] has bit b set when body b is body k
  // or one of its ancestors (on the device a per-block LDS table, chainMasks)
  const unsigned long long* chain;
  // cooperative constraint kernel only (else nullptr; it runs only when nv <= 64): dchain[k]
  // has bit j set when dof j belongs to body k or one of its ancestors (a per-block LDS table)
  const unsigned long long* dchain;
  // geom positions as collision reads them: geom_xpos itself, or (gstage) a per-lane LDS
  // copy that collision() fills first -- the broadphase reads every candidate pair's
  // positions, and LDS turns those loads from memory round trips into LDS latency
  SP<S> gxpos;
  bool gstage;
  // the static collision program (csrc/pair_program.h: candidate geom pairs in the order the
  // serial mj_collision emits contacts, midphase sort and predefined pairs included) with each
  // entry's predefined-pair index (-1 for a swept pair); nullptr: collision() walks the body
  // pairs itself
  const CoopPair* prog;
  const int* prog_ipair;
  int nprog;
  // cooperative constraint kernel only (else nullptr), per-instance LDS copies: cdq[8*j+c]
  // holds cdof (c < 6), qvel (c = 6) and qacc (c = 7) of dof j for the contact rows; fst[r]
  // receives efc_force[r] as a row is finished, for the J'force pass
  const double* cdq;
  double* fst;
  int nfst;                                  // rows r < nfst have fst[r]
  // cooperative constraint kernel only (else nullptr): per contact, its bodies and their
  // roots (b1, b2, body_rootid[b1], body_rootid[b2]) in LDS, written with the contact, for
  // contacts i < ncbody
  const int* cbody;
  int ncbody;
  // the native solver's scratch (the ccd / ccdi fields) seen per lane: the lane's contiguous
  // slice of the field's block storage, so a polytope vertex (9 doubles) or face (4 doubles,
  // 7 ints) is one or two cache lines of its own rather than one line per component shared
  // with lanes that are elsewhere in their iterations
  double* ccdx;
  int* ccdxi;
};

// chain[k] for body k (the fused path's ancestor test, one bit per body)
MJH_HD unsigned long long chainMask(const mjhipModel& m, int k) {
  unsigned long long mk = 0;
  for (int b = k; b > 0; b = m.body_parentid[b]) mk |= 1ull << b;
  return mk;
}

// whether mj_inverseSkip(skipstage) can take the fused constraint path
MJH_HD bool fusedOk(const mjhipModel& m, int skipstage) {
  return skipstage == mjhipSTAGE_NONE && !(m.opt.enableflags & mjhipENBL_INVDISCRETE) &&
         !mjh_isSparse(&m) &&
         m.nbody <= 64 && (m.ngeom <= 64 || !mjhip_contactsEnabled(&m)) &&
         !(m.opt.cone == mjhipCONE_ELLIPTIC && mjhip_contactsEnabled(&m));
}

// dynamic LDS of a fused contact kernel: the per-lane geom position copy (Lane::gxpos)
MJH_HD unsigned gstageBytes(const mjhipModel& m) { return 3u*m.ngeom*64*sizeof(double); }

//---------------------------------- engine_util_blas.c ---------------------------------------

template <class R> MJH_HD void zero3(R r) { r[0] = 0; r[1] = 0; r[2] = 0; }
template <class R, class A> MJH_HD void copy3(R r, A a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
template <class R, class A> MJH_HD void copy4(R r, A a) {
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
}
template <class R, class A> MJH_HD void scl3(R r, A a, double s) {
  r[0] = a[0]*s; r[1] = a[1]*s; r[2] = a[2]*s;
}
template <class R, class A, class B> MJH_HD void add3(R r, A a, B b) {
  r[0] = a[0]+b[0]; r[1] = a[1]+b[1]; r[2] = a[2]+b[2];
}
template <class R, class A, class B> MJH_HD void sub3(R r, A a, B b) {
  r[0] = a[0]-b[0]; r[1] = a[1]-b[1]; r[2] = a[2]-b[2];
}
template <class R, class A> MJH_HD void addTo3(R r, A a) {
  r[0] += a[0]; r[1] += a[1]; r[2] += a[2];
}
template <class R, class A> MJH_HD void addToScl3(R r, A a, double s) {
  r[0] += a[0]*s; r[1] += a[1]*s; r[2] += a[2]*s;
}
template <class R, class A, class B> MJH_HD void cross(R r, A a, B b) {
  double t0 = a[1]*b[2] - a[2]*b[1], t1 = a[2]*b[0] - a[0]*b[2], t2 = a[0]*b[1] - a[1]*b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <class R> MJH_HD void zero(R r, int n) { for (int i = 0; i < n; i++) r[i] = 0; }
template <class R, class A> MJH_HD void copy(R r, A a, int n) {
  for (int i = 0; i < n; i++) r[i] = a[i];
}
// a value barrier: r[0..n) stay the rounded values computed, so no later multiply-add is
// contracted or re-associated through them. The straight-line va stage and the acceleration
// stage alone (codegen.py _gen_acc) pin the same shared terms of their RNE recursion, so the
// two round identically whatever the compiler fuses in either (mjd_inverseFD's k_accskip).
template <class R> MJH_HD void pin(R r, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  for (int i = 0; i < n; i++) __asm__("" : "+v"(r[i]));
#endif
}
template <class R, class A> MJH_HD void scl(R r, A a, double s, int n) {
  for (int i = 0; i < n; i++) r[i] = a[i]*s;
}
template <class R, class A, class B> MJH_HD void add(R r, A a, B b, int n) {
  for (int i = 0; i < n; i++) r[i] = a[i] + b[i];
}
template <class R, class A> MJH_HD void addTo(R r, A a, int n) {
  for (int i = 0; i < n; i++) r[i] += a[i];
}
template <class R, class A> MJH_HD void subFrom(R r, A a, int n) {
  for (int i = 0; i < n; i++) r[i] -= a[i];
}
template <class R, class A> MJH_HD void addToScl(R r, A a, double s, int n) {
  for (int i = 0; i < n; i++) r[i] += a[i]*s;
}

// engine_util_blas.c:123-140
template <class V> MJH_HD double normalize3(V v) {
  double norm = sqrt(v[0]*v[0] + v[1]*v[1] + v[2]*v[2]);
  if (norm < MINVAL) {
    v[0] = 1; v[1] = 0; v[2] = 0;
  } else {
    double normInv = 1/norm;
    v[0] *= normInv; v[1] *= normInv; v[2] *= normInv;
  }
  return norm;
}

// engine_util_blas.c:269-285
template <class V> MJH_HD double normalize4(V v) {
  double norm = sqrt(v[0]*v[0] + v[1]*v[1] + v[2]*v[2] + v[3]*v[3]);
  if (norm < MINVAL) {
    v[0] = 1; v[1] = 0; v[2] = 0; v[3] = 0;
  } else if (fabs(norm - 1) > MINVAL) {
    double normInv = 1/norm;
    v[0] *= normInv; v[1] *= normInv; v[2] *= normInv; v[3] *= normInv;
  }
  return norm;
}

// Branch-free forms of addToScl-if-nonzero / normalize3 / normalize4 for the generated
// kernels. Results are identical to the branching forms (same operations, selected). A
// straight-line body without branches is one scheduling region, so the compiler cannot sink
// computation into later basic blocks, away from the loads the kernel prefetched for it.
template <class R, class A> MJH_HD void addToSclIf(R r, A a, double s, int n) {
  for (int i = 0; i < n; i++) {
    double t = r[i] + a[i]*s;
    r[i] = s ? t : r[i];
  }
}

template <class V> MJH_HD double normalize3s(V v) {
  double norm = sqrt(v[0]*v[0] + v[1]*v[1] + v[2]*v[2]);
  bool small = norm < MINVAL;
  double normInv = 1/norm;
  double a0 = v[0]*normInv, a1 = v[1]*normInv, a2 = v[2]*normInv;
  v[0] = small ? 1.0 : a0; v[1] = small ? 0.0 : a1; v[2] = small ? 0.0 : a2;
  return norm;
}

template <class V> MJH_HD double normalize4s(V v) {
  double norm = sqrt(v[0]*v[0] + v[1]*v[1] + v[2]*v[2] + v[3]*v[3]);
  bool small = norm < MINVAL;
  bool scale = !small && fabs(norm - 1) > MINVAL;
  double normInv = 1/norm;
  double a0 = v[0]*normInv, a1 = v[1]*normInv, a2 = v[2]*normInv, a3 = v[3]*normInv;
  v[0] = small ? 1.0 : (scale ? a0 : v[0]);
  v[1] = small ? 0.0 : (scale ? a1 : v[1]);
  v[2] = small ? 0.0 : (scale ? a2 : v[2]);
  v[3] = small ? 0.0 : (scale ? a3 : v[3]);
  return norm;
}

// engine_util_blas.c:165-176
template <class R, class M, class V> MJH_HD void mulMatVec3(R res, M mat, V vec) {
  double t0 = mat[0]*vec[0] + mat[1]*vec[1] + mat[2]*vec[2];
  double t1 = mat[3]*vec[0] + mat[4]*vec[1] + mat[5]*vec[2];
  double t2 = mat[6]*vec[0] + mat[7]*vec[1] + mat[8]*vec[2];
  res[0] = t0; res[1] = t1; res[2] = t2;
}

// engine_util_blas.c:680-741 (scalar branch): lanes 0..3, (r0+r2)+(r1+r3), then the tail
template <class A, class B> MJH_HD double dot(A a, B b, int n) {
  int i = 0, n_4 = n - 4;
  double r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  for (; i <= n_4; i += 4) {
    r0 += a[i]*b[i];
    r1 += a[i+1]*b[i+1];
    r2 += a[i+2]*b[i+2];
    r3 += a[i+3]*b[i+3];
  }
  double res = (r0 + r2) + (r1 + r3);
  int n_i = n - i;
  if (n_i == 3) {
    res += a[i]*b[i] + a[i+1]*b[i+1] + a[i+2]*b[i+2];
  } else if (n_i == 2) {
    res += a[i]*b[i] + a[i+1]*b[i+1];
  } else if (n_i == 1) {
    res += a[i]*b[i];
  }
  return res;
}

// mju_dot for n = 6 (the spatial-vector case): ((p0+p2)+(p1+p3)) + (p4+p5)
template <class A, class B> MJH_HD double dot6(A a, B b) {
  double r0 = a[0]*b[0], r1 = a[1]*b[1], r2 = a[2]*b[2], r3 = a[3]*b[3];
  double res = (r0 + r2) + (r1 + r3);
  res += a[4]*b[4] + a[5]*b[5];
  return res;
}

// engine_util_blas.c:756-766
template <class R, class M, class V> MJH_HD void mulMatTVec(R res, M mat, V vec, int nr, int nc) {
  zero(res, nc);
  for (int r = 0; r < nr; r++) {
    double tmp = vec[r];
    if (tmp) addToScl(res, mat + r*nc, tmp, nc);
  }
}

// engine_util_sparse.h:115-160 (scalar branch; the AVX branch, engine_util_sparse_avx.h:34-
// 105, groups the products the same way)
template <class V1, class V2, class I> MJH_HD double dotSparse(V1 v1, V2 v2, int nnz1, I ind1) {
  int i = 0, n_4 = nnz1 - 4;
  double r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  for (; i <= n_4; i += 4) {
    r0 += v1[i+0]*v2[ind1[i+0]];
    r1 += v1[i+1]*v2[ind1[i+1]];
    r2 += v1[i+2]*v2[ind1[i+2]];
    r3 += v1[i+3]*v2[ind1[i+3]];
  }
  double res = (r0 + r2) + (r1 + r3);
  for (; i < nnz1; i++) res += v1[i]*v2[ind1[i]];
  return res;
}

//---------------------------------- engine_util_spatial.c ------------------------------------

// :23-46
template <class R, class V, class Q> MJH_HD void rotVecQuat(R res, V vec, Q quat) {
  if (vec[0] == 0 && vec[1] == 0 && vec[2] == 0) {
    zero3(res);
  } else if (quat[0] == 1 && quat[1] == 0 && quat[2] == 0 && quat[3] == 0) {
    copy3(res, vec);
  } else {
    double t0 = quat[0]*vec[0] + quat[2]*vec[2] - quat[3]*vec[1];
    double t1 = quat[0]*vec[1] + quat[3]*vec[0] - quat[1]*vec[2];
    double t2 = quat[0]*vec[2] + quat[1]*vec[1] - quat[2]*vec[0];
    double r0 = vec[0] + 2 * (quat[2]*t2 - quat[3]*t1);
    double r1 = vec[1] + 2 * (quat[3]*t0 - quat[1]*t2);
    double r2 = vec[2] + 2 * (quat[1]*t1 - quat[2]*t0);
    res[0] = r0; res[1] = r1; res[2] = r2;
  }
}

// :62-74
template <class R, class A, class B> MJH_HD void mulQuat(R res, A qa, B qb) {
  double t0 = qa[0]*qb[0] - qa[1]*qb[1] - qa[2]*qb[2] - qa[3]*qb[3];
  double t1 = qa[0]*qb[1] + qa[1]*qb[0] + qa[2]*qb[3] - qa[3]*qb[2];
  double t2 = qa[0]*qb[2] - qa[1]*qb[3] + qa[2]*qb[0] + qa[3]*qb[1];
  double t3 = qa[0]*qb[3] + qa[1]*qb[2] - qa[2]*qb[1] + qa[3]*qb[0];
  res[0] = t0; res[1] = t1; res[2] = t2; res[3] = t3;
}

// :97-114
template <class R, class A> MJH_HD void axisAngle2Quat(R res, A axis, double angle) {
  if (angle == 0) {
    res[0] = 1; res[1] = 0; res[2] = 0; res[3] = 0;
  } else {
    double s = sin(angle*0.5);
    res[0] = cos(angle*0.5);
    res[1] = axis[0]*s;
    res[2] = axis[1]*s;
    res[3] = axis[2]*s;
  }
}

// axisAngle2Quat with s = sin(angle/2), c = cos(angle/2) computed elsewhere, as selects
template <class R, class A> MJH_HD void axisAngle2QuatSC(R res, A axis, double angle, double s,
                                                         double c) {
  const bool z = angle == 0;
  res[0] = z ? 1.0 : c;
  res[1] = z ? 0.0 : axis[0]*s;
  res[2] = z ? 0.0 : axis[1]*s;
  res[3] = z ? 0.0 : axis[2]*s;
}

// :119-133
template <class R, class Q> MJH_HD void quat2Vel(R res, Q quat, double dt) {
  double axis[3] = {quat[1], quat[2], quat[3]};
  double sin_a_2 = normalize3(axis);
  double speed = 2 * atan2(sin_a_2, quat[0]);
  if (speed > mjhipPI) speed -= 2*mjhipPI;
  speed /= dt;
  scl3(res, axis, speed);
}

// :138-146
template <class R, class A, class B> MJH_HD void subQuat(R res, A qa, B qb) {
  double qneg[4] = {qb[0], -qb[1], -qb[2], -qb[3]}, qdif[4];
  mulQuat(qdif, qneg, qa);
  quat2Vel(res, qdif, 1);
}

// :151-187
template <class R, class Q> MJH_HD void quat2Mat(R res, Q quat) {
  if (quat[0] == 1 && quat[1] == 0 && quat[2] == 0 && quat[3] == 0) {
    res[0] = 1; res[1] = 0; res[2] = 0;
    res[3] = 0; res[4] = 1; res[5] = 0;
    res[6] = 0; res[7] = 0; res[8] = 1;
  } else {
    const double q00 = quat[0]*quat[0], q01 = quat[0]*quat[1], q02 = quat[0]*quat[2];
    const double q03 = quat[0]*quat[3], q11 = quat[1]*quat[1], q12 = quat[1]*quat[2];
    const double q13 = quat[1]*quat[3], q22 = quat[2]*quat[2], q23 = quat[2]*quat[3];
    const double q33 = quat[3]*quat[3];
    res[0] = q00 + q11 - q22 - q33;
    res[4] = q00 - q11 + q22 - q33;
    res[8] = q00 - q11 - q22 + q33;
    res[1] = 2*(q12 - q03);
    res[2] = 2*(q13 + q02);
    res[3] = 2*(q12 + q03);
    res[5] = 2*(q23 - q01);
    res[6] = 2*(q13 - q02);
    res[7] = 2*(q23 + q01);
  }
}

// quat2Mat with the identity test as selects (generated kernels; see normalize4s)
template <class R, class Q> MJH_HD void quat2Mats(R res, Q quat) {
  const bool id = quat[0] == 1 && quat[1] == 0 && quat[2] == 0 && quat[3] == 0;
  const double q00 = quat[0]*quat[0], q01 = quat[0]*quat[1], q02 = quat[0]*quat[2];
  const double q03 = quat[0]*quat[3], q11 = quat[1]*quat[1], q12 = quat[1]*quat[2];
  const double q13 = quat[1]*quat[3], q22 = quat[2]*quat[2], q23 = quat[2]*quat[3];
  const double q33 = quat[3]*quat[3];
  const double r0 = q00 + q11 - q22 - q33, r4 = q00 - q11 + q22 - q33;
  const double r8 = q00 - q11 - q22 + q33;
  const double r1 = 2*(q12 - q03), r2 = 2*(q13 + q02), r3 = 2*(q12 + q03);
  const double r5 = 2*(q23 - q01), r6 = 2*(q13 - q02), r7 = 2*(q23 + q01);
  res[0] = id ? 1.0 : r0; res[1] = id ? 0.0 : r1; res[2] = id ? 0.0 : r2;
  res[3] = id ? 0.0 : r3; res[4] = id ? 1.0 : r4; res[5] = id ? 0.0 : r5;
  res[6] = id ? 0.0 : r6; res[7] = id ? 0.0 : r7; res[8] = id ? 1.0 : r8;
}

// :385-396
template <class R, class A, class B> MJH_HD void crossMotion(R res, A vel, B v) {
  double r0 = -vel[2]*v[1] + vel[1]*v[2];
  double r1 =  vel[2]*v[0] - vel[0]*v[2];
  double r2 = -vel[1]*v[0] + vel[0]*v[1];
  double r3 = -vel[2]*v[4] + vel[1]*v[5];
  double r4 =  vel[2]*v[3] - vel[0]*v[5];
  double r5 = -vel[1]*v[3] + vel[0]*v[4];
  r3 += -vel[5]*v[1] + vel[4]*v[2];
  r4 +=  vel[5]*v[0] - vel[3]*v[2];
  r5 += -vel[4]*v[0] + vel[3]*v[1];
  res[0] = r0; res[1] = r1; res[2] = r2; res[3] = r3; res[4] = r4; res[5] = r5;
}

// :401-412
template <class R, class A, class B> MJH_HD void crossForce(R res, A vel, B f) {
  double r0 = -vel[2]*f[1] + vel[1]*f[2];
  double r1 =  vel[2]*f[0] - vel[0]*f[2];
  double r2 = -vel[1]*f[0] + vel[0]*f[1];
  double r3 = -vel[2]*f[4] + vel[1]*f[5];
  double r4 =  vel[2]*f[3] - vel[0]*f[5];
  double r5 = -vel[1]*f[3] + vel[0]*f[4];
  r0 += -vel[5]*f[4] + vel[4]*f[5];
  r1 +=  vel[5]*f[3] - vel[3]*f[5];
  r2 += -vel[4]*f[3] + vel[3]*f[4];
  res[0] = r0; res[1] = r1; res[2] = r2; res[3] = r3; res[4] = r4; res[5] = r5;
}

// :417-447
template <class R, class I, class M, class D>
MJH_HD void inertCom(R res, I inert, M mat, D dif, double mass) {
  double tmp[9] = {mat[0]*inert[0], mat[3]*inert[0], mat[6]*inert[0],
                   mat[1]*inert[1], mat[4]*inert[1], mat[7]*inert[1],
                   mat[2]*inert[2], mat[5]*inert[2], mat[8]*inert[2]};
  double r0 = mat[0]*tmp[0] + mat[1]*tmp[3] + mat[2]*tmp[6];
  double r1 = mat[3]*tmp[1] + mat[4]*tmp[4] + mat[5]*tmp[7];
  double r2 = mat[6]*tmp[2] + mat[7]*tmp[5] + mat[8]*tmp[8];
  double r3 = mat[0]*tmp[1] + mat[1]*tmp[4] + mat[2]*tmp[7];
  double r4 = mat[0]*tmp[2] + mat[1]*tmp[5] + mat[2]*tmp[8];
  double r5 = mat[3]*tmp[2] + mat[4]*tmp[5] + mat[5]*tmp[8];
  r0 += mass*(dif[1]*dif[1] + dif[2]*dif[2]);
  r1 += mass*(dif[0]*dif[0] + dif[2]*dif[2]);
  r2 += mass*(dif[0]*dif[0] + dif[1]*dif[1]);
  r3 -= mass*dif[0]*dif[1];
  r4 -= mass*dif[0]*dif[2];
  r5 -= mass*dif[1]*dif[2];
  res[0] = r0; res[1] = r1; res[2] = r2; res[3] = r3; res[4] = r4; res[5] = r5;
  res[6] = mass*dif[0];
  res[7] = mass*dif[1];
  res[8] = mass*dif[2];
  res[9] = mass;
}

// :452-459
template <class R, class I, class V> MJH_HD void mulInertVec(R res, I i, V v) {
  double r0 = i[0]*v[0] + i[3]*v[1] + i[4]*v[2] - i[8]*v[4] + i[7]*v[5];
  double r1 = i[3]*v[0] + i[1]*v[1] + i[5]*v[2] + i[8]*v[3] - i[6]*v[5];
  double r2 = i[4]*v[0] + i[5]*v[1] + i[2]*v[2] - i[7]*v[3] + i[6]*v[4];
  double r3 = i[8]*v[1] - i[7]*v[2] + i[9]*v[3];
  double r4 = i[6]*v[2] - i[8]*v[0] + i[9]*v[4];
  double r5 = i[7]*v[0] - i[6]*v[1] + i[9]*v[5];
  res[0] = r0; res[1] = r1; res[2] = r2; res[3] = r3; res[4] = r4; res[5] = r5;
}

// :464-476 (hinge/ball: offset given)
template <class R, class A, class O> MJH_HD void dofComHinge(R res, A axis, O offset) {
  copy3(res, axis);
  cross(res + 3, axis, offset);
}

// :481-489
template <class R, class D, class V> MJH_HD void mulDofVec(R res, D dof, V vec, int n) {
  if (n == 1) {
    scl(res, dof, vec[0], 6);
  } else if (n <= 0) {
    zero(res, 6);
  } else {
    mulMatTVec(res, dof, vec, n, 6);
  }
}

// mju_quatIntegrate :241-250
template <class Q, class V> MJH_HD void quatIntegrate(Q quat, V vel, double scale) {
  double tmp[3] = {vel[0], vel[1], vel[2]}, qrot[4];
  double angle = scale * normalize3(tmp);
  axisAngle2Quat(qrot, tmp, angle);
  normalize4(quat);
  mulQuat(quat, quat, qrot);
}

//---------------------------------- engine_support.c -----------------------------------------

// mj_local2Global :1565-1606 (pos and quat both given)
template <int S, class P, class Q>
MJH_HD void local2Global(const Lane<S>& d, SP<S> xpos, SP<S> xmat, P pos, Q quat, int body,
                         int sameframe) {
  switch (sameframe) {
  case mjhipSAMEFRAME_NONE:
  case mjhipSAMEFRAME_BODYROT:
  case mjhipSAMEFRAME_INERTIAROT:
    mulMatVec3(xpos, d.xmat + 9*body, pos);
    addTo3(xpos, d.xpos + 3*body);
    break;
  case mjhipSAMEFRAME_BODY:
    copy3(xpos, d.xpos + 3*body);
    break;
  case mjhipSAMEFRAME_INERTIA:
    copy3(xpos, d.xipos + 3*body);
    break;
  }
  double tmp[4];
  switch (sameframe) {
  case mjhipSAMEFRAME_NONE:
    mulQuat(tmp, d.xquat + 4*body, quat);
    quat2Mat(xmat, tmp);
    break;
  case mjhipSAMEFRAME_BODY:
  case mjhipSAMEFRAME_BODYROT:
    copy(xmat, d.xmat + 9*body, 9);
    break;
  case mjhipSAMEFRAME_INERTIA:
  case mjhipSAMEFRAME_INERTIAROT:
    copy(xmat, d.ximat + 9*body, 9);
    break;
  }
}

// mj_jac :389-441 (dense), into jacp / jacr
template <int S, class P>
MJH_HD void jacInto(const mjhipModel& m, const Lane<S>& d, SP<S> jacp, SP<S> jacr, P point,
                    int body) {
  int nv = m.nv;
  double offset[3];
  zero(jacp, 3*nv);
  zero(jacr, 3*nv);
  sub3(offset, point, d.subtree_com + 3*m.body_rootid[body]);
  while (body && !m.body_dofnum[body]) body = m.body_parentid[body];
  if (!body) return;
  int i = m.body_dofadr[body] + m.body_dofnum[body] - 1;
  while (i >= 0) {
    SP<S> cdof = d.cdof + 6*i;
    jacr[i+0*nv] = cdof[0];
    jacr[i+1*nv] = cdof[1];
    jacr[i+2*nv] = cdof[2];
    double tmp[3];
    cross(tmp, cdof, offset);
    jacp[i+0*nv] = cdof[3] + tmp[0];
    jacp[i+1*nv] = cdof[4] + tmp[1];
    jacp[i+2*nv] = cdof[5] + tmp[2];
    i = m.dof_parentid[i];
  }
}

template <int S, class P>
MJH_HD void jac(const mjhipModel& m, const Lane<S>& d, P point, int body) {
  jacInto(m, d, d.jacp, d.jacr, point, body);
}


//---------------------------------- engine_collision_*.c -------------------------------------
// mj_collision for the primitive pairs (the static candidate rules are in
// include/mjhip_contact.h; the oracle restates the reference's broadphase on its own, so the
// parity tests check these rules against it); contacts go to the con_* scratch fields.

struct RawContact { double dist, pos[3], frame[9]; };

template <class A, class B> MJH_HD double dot3(A a, B b) { return a[0]*b[0] + a[1]*b[1] + a[2]*b[2]; }
MJH_HD double clip(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

// c[k] = t for k = 0 or 1 as value selects on constant indices (a store through a selected
// pointer would keep c in private memory)
MJH_HD void putRaw(RawContact* c, int k, const RawContact& t) {
  const bool z = k == 0;
  c[0].dist = z ? t.dist : c[0].dist;
  c[1].dist = z ? c[1].dist : t.dist;
  for (int j = 0; j < 3; j++) {
    c[0].pos[j] = z ? t.pos[j] : c[0].pos[j];
    c[1].pos[j] = z ? c[1].pos[j] : t.pos[j];
  }
  for (int j = 0; j < 9; j++) {
    c[0].frame[j] = z ? t.frame[j] : c[0].frame[j];
    c[1].frame[j] = z ? c[1].frame[j] : t.frame[j];
  }
}

// engine_collision_primitive.c:95-195 mjc_PlaneCylinder; each contact goes to emit() as it
// is made (up to 4), so no contact array is kept
template <class P1, class M1, class P2, class M2, class E>
MJH_HD void colPlaneCylinder(double margin, P1 pos1, M1 mat1, P2 pos2, M2 mat2,
                             const double* size2, E&& emit) {
  double normal[3] = {mat1[2], mat1[5], mat1[8]};
  double axis[3] = {mat2[2], mat2[5], mat2[8]};
  double prjaxis = dot3(normal, axis);
  if (prjaxis > 0) {
    scl3(axis, axis, -1);
    prjaxis = -prjaxis;
  }
  double vec[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
  const double dist0 = dot3(vec, normal);
  scl3(vec, axis, prjaxis);
  vec[0] -= normal[0]; vec[1] -= normal[1]; vec[2] -= normal[2];
  const double len_sqr = dot3(vec, vec);
  if (len_sqr >= MINVAL*MINVAL) {
    const double scl = size2[0]/sqrt(len_sqr);
    vec[0] *= scl; vec[1] *= scl; vec[2] *= scl;
  } else {
    vec[0] = mat2[0]*size2[0];
    vec[1] = mat2[3]*size2[0];
    vec[2] = mat2[6]*size2[0];
  }
  const double prjvec = dot3(vec, normal);
  scl3(axis, axis, size2[1]);
  prjaxis *= size2[1];
  RawContact c;
  for (int k = 0; k < 3; k++) c.frame[k] = normal[k];
  c.frame[3] = 0; c.frame[4] = 0; c.frame[5] = 0;
  for (int k = 6; k < 9; k++) c.frame[k] = 0;
  if (!(dist0 + prjaxis + prjvec <= margin)) return;
  c.dist = dist0 + prjaxis + prjvec;
  add3(c.pos, pos2, vec);
  addTo3(c.pos, axis);
  addToScl3(c.pos, normal, -c.dist*0.5);
  if (!emit(c)) return;
  if (dist0 - prjaxis + prjvec <= margin) {
    c.dist = dist0 - prjaxis + prjvec;
    add3(c.pos, pos2, vec);
    c.pos[0] -= axis[0]; c.pos[1] -= axis[1]; c.pos[2] -= axis[2];
    addToScl3(c.pos, normal, -c.dist*0.5);
    if (!emit(c)) return;
  }
  const double prjvec1 = -prjvec*0.5;
  if (dist0 + prjaxis + prjvec1 <= margin) {
    double vec1[3];
    cross(vec1, vec, axis);
    normalize3(vec1);
    scl3(vec1, vec1, size2[0]*sqrt(3.0)/2);
    c.dist = dist0 + prjaxis + prjvec1;
    add3(c.pos, pos2, vec1);
    addTo3(c.pos, axis);
    addToScl3(c.pos, vec, -0.5);
    addToScl3(c.pos, normal, -c.dist*0.5);
    if (!emit(c)) return;
    c.dist = dist0 + prjaxis + prjvec1;
    sub3(c.pos, pos2, vec1);
    addTo3(c.pos, axis);
    addToScl3(c.pos, vec, -0.5);
    addToScl3(c.pos, normal, -c.dist*0.5);
    emit(c);
  }
}

// engine_collision_primitive.c:200-243 mjc_PlaneBox: the (up to 4) lowest corners
template <class P1, class M1, class P2, class M2, class E>
MJH_HD void colPlaneBox(double margin, P1 pos1, M1 mat1, P2 pos2, M2 mat2, const double* size2,
                        E&& emit) {
  const double norm[3] = {mat1[2], mat1[5], mat1[8]};
  const double dif[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
  const double dist = dot3(dif, norm);
  RawContact c;
  for (int k = 0; k < 3; k++) c.frame[k] = norm[k];
  for (int k = 3; k < 9; k++) c.frame[k] = 0;
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    double vec[3] = {(i&1) ? size2[0] : -size2[0], (i&2) ? size2[1] : -size2[1],
                     (i&4) ? size2[2] : -size2[2]};
    double corner[3];
    mulMatVec3(corner, mat2, vec);
    const double ldist = dot3(norm, corner);
    if (dist + ldist > margin || ldist > 0) continue;
    c.dist = dist + ldist;
    addTo3(corner, pos2);
    scl3(vec, norm, -c.dist/2);
    add3(c.pos, corner, vec);
    if (!emit(c) || ++cnt >= 4) return;
  }
}

// engine_collision_primitive.c mjraw_PlaneSphere
template <class P1, class M1, class P2>
MJH_HD int rawPlaneSphere(RawContact* c, double margin, P1 pos1, M1 mat1, P2 pos2, double r2) {
  c->frame[0] = mat1[2];
  c->frame[1] = mat1[5];
  c->frame[2] = mat1[8];
  double tmp[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
  double cdist = dot3(tmp, c->frame);
  if (cdist > margin + r2) return 0;
  c->dist = cdist - r2;
  scl3(tmp, c->frame, -c->dist/2 - r2);
  add3(c->pos, pos2, tmp);
  zero3(c->frame + 3);
  return 1;
}

// mjc_PlaneCapsule
template <class P1, class M1, class P2, class M2>
MJH_HD int colPlaneCapsule(RawContact* c, double margin, P1 pos1, M1 mat1, P2 pos2, M2 mat2,
                           const double* size2) {
  double axis[3] = {mat2[2], mat2[5], mat2[8]};
  double seg[3] = {size2[1]*axis[0], size2[1]*axis[1], size2[1]*axis[2]};
  double p[3];
  RawContact t;
  add3(p, pos2, seg);
  int n = rawPlaneSphere(&t, margin, pos1, mat1, p, size2[0]);
  copy3(t.frame + 3, axis);
  if (n) putRaw(c, 0, t);
  sub3(p, pos2, seg);
  int n2 = rawPlaneSphere(&t, margin, pos1, mat1, p, size2[0]);
  copy3(t.frame + 3, axis);
  if (n2) putRaw(c, n, t);
  return n + n2;
}

// mjraw_SphereSphere
template <class P1, class M1, class P2, class M2>
MJH_HD int rawSphereSphere(RawContact* c, double margin, P1 pos1, M1 mat1, double r1, P2 pos2,
                           M2 mat2, double r2) {
  double dif[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
  double cdist_sqr = dot3(dif, dif);
  double min_dist = margin + r1 + r2;
  if (cdist_sqr > min_dist*min_dist) return 0;
  c->dist = sqrt(cdist_sqr) - r1 - r2;
  sub3(c->frame, pos2, pos1);
  double len = normalize3(c->frame);
  if (len < MINVAL) {
    double a1[3] = {mat1[2], mat1[5], mat1[8]}, a2[3] = {mat2[2], mat2[5], mat2[8]};
    cross(c->frame, a1, a2);
    normalize3(c->frame);
  }
  scl3(c->pos, c->frame, r1 + c->dist/2);
  addTo3(c->pos, pos1);
  zero3(c->frame + 3);
  return 1;
}

template <class R, class M, class V> MJH_HD void mulMatTVec3(R res, M mat, V vec);

// engine_collision_box.c:38-92 mjraw_SphereBox (the box's size clamps the sphere centre)
template <class P1, class P2, class M2>
MJH_HD int rawSphereBox(RawContact* c, double margin, P1 pos1, double r1, P2 pos2, M2 mat2,
                        const double* size2) {
  double tmp[3], center[3], clamped[3], deepest[3], pos[3];
  sub3(tmp, pos1, pos2);
  mulMatTVec3(center, mat2, tmp);
  copy3(clamped, center);
  for (int i = 0; i < 3; i++) {        // mju_clampVec
    if (size2[i] > 0) {
      if (clamped[i] < -size2[i]) clamped[i] = -size2[i];
      else if (clamped[i] > size2[i]) clamped[i] = size2[i];
    }
  }
  copy3(deepest, center);
  sub3(tmp, clamped, center);
  double dist = normalize3(tmp);
  if (dist - r1 > margin) return 0;
  if (dist <= MINVAL) {                 // centre inside the box: nearest face
    double closest = (size2[0] + size2[1] + size2[2])*2;
    int k = 0;
    for (int i = 0; i < 6; i++) {
      const double f = fabs((i % 2 ? 1 : -1)*size2[i/2] - center[i/2]);
      if (closest > f) { closest = f; k = i; }
    }
    double nearest[3] = {0, 0, 0};
    nearest[k/2] = (k % 2 ? -1 : 1);
    copy3(pos, center);
    addToScl3(pos, nearest, (r1 - closest)/2);
    mulMatVec3(c->frame, mat2, nearest);
    dist = -closest;
  } else {
    addToScl3(deepest, tmp, r1);
    zero3(pos);
    addToScl3(pos, clamped, 0.5);
    addToScl3(pos, deepest, 0.5);
    mulMatVec3(c->frame, mat2, tmp);
  }
  mulMatVec3(tmp, mat2, pos);
  add3(c->pos, tmp, pos2);
  c->dist = dist - r1;
  zero3(c->frame + 3);
  return 1;
}

// mjraw_SphereCapsule
template <class P1, class M1, class P2, class M2>
MJH_HD int colSphereCapsule(RawContact* c, double margin, P1 pos1, M1 mat1, double r1, P2 pos2,
                            M2 mat2, const double* size2) {
  double len = size2[1];
  double axis[3] = {mat2[2], mat2[5], mat2[8]};
  double vec[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
  double x = clip(dot3(axis, vec), -len, len);
  scl3(vec, axis, x);
  addTo3(vec, pos2);
  return rawSphereSphere(c, margin, pos1, mat1, r1, vec, mat2, size2[0]);
}

// mjc_SphereCylinder (engine_collision_primitive.c:323-391): side (sphere-sphere with the
// axis point), cap (plane-sphere on the cap plane, normal flipped) or rim corner (sphere-
// sphere with a point sphere at the corner)
template <class P1, class M1, class P2, class M2>
MJH_HD int colSphereCylinder(RawContact* c, double margin, P1 pos1, M1 mat1, double r1,
                             P2 pos2, M2 mat2, const double* size2) {
  const double radius = size2[0], height = size2[1];
  double axis[3] = {mat2[2], mat2[5], mat2[8]};
  double vec[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
  const double x = dot3(axis, vec);
  double a_proj[3], p_proj[3];
  scl3(a_proj, axis, x);
  sub3(p_proj, vec, a_proj);
  const double p_proj_sqr = dot3(p_proj, p_proj);
  bool collide_side = fabs(x) < height;
  bool collide_cap = p_proj_sqr < radius*radius;
  if (collide_side && collide_cap) {
    const double dist_cap = height - fabs(x);
    const double dist_radius = radius - sqrt(p_proj_sqr);
    if (dist_cap < dist_radius) {
      collide_side = false;
    } else {
      collide_cap = false;
    }
  }
  if (collide_side) {
    addTo3(a_proj, pos2);
    return rawSphereSphere(c, margin, pos1, mat1, r1, a_proj, mat2, size2[0]);
  }
  if (collide_cap) {
    double mcap[9], pos_cap[3];
    const double sgn = x > 0 ? 1.0 : -1.0;
    for (int k = 0; k < 9; k++) mcap[k] = mat2[k];
    if (x <= 0) {                       // bottom cap: the flipped frame
      for (int r = 0; r < 3; r++) {
        mcap[3*r] = -mat2[3*r];
        mcap[3*r+2] = -mat2[3*r+2];
      }
    }
    for (int k = 0; k < 3; k++) pos_cap[k] = pos2[k] + (sgn*height)*axis[k];
    const int ncon = rawPlaneSphere(c, margin, pos_cap, mcap, pos1, r1);
    if (ncon) {
      for (int k = 0; k < 3; k++) c->frame[k] = c->frame[k]*-1;
    }
    return ncon;
  }
  scl3(p_proj, p_proj, size2[0] / sqrt(p_proj_sqr));
  scl3(vec, axis, x > 0 ? height : -height);
  addTo3(vec, p_proj);
  addTo3(vec, pos2);
  return rawSphereSphere(c, margin, pos1, mat1, r1, vec, mat2, 0.0);
}

// mjraw_CapsuleBox (engine_collision_box.c:121-594): the box feature closest to the capsule
// segment (an end point against a face, or the segment against one of the 12 edges, in the
// box frame), the second point along the segment that can still touch the box, then one
// sphere-box contact of the capsule's radius at each point (at most 2). The reference's
// j == 2 block inside the edge loop computes nothing that is used later; it is omitted.
template <class P1, class M1, class P2, class M2>
MJH_HD int colCapsuleBox(RawContact* c, double margin, P1 pos1, M1 mat1, const double* size1,
                         P2 pos2, M2 mat2, const double* size2) {
  double tmp[3], pos[3], axis[3], halfaxis[3];
  const double hl = size1[1];
  sub3(tmp, pos1, pos2);
  mulMatTVec3(pos, mat2, tmp);
  const double a1[3] = {mat1[2], mat1[5], mat1[8]};
  mulMatTVec3(axis, mat2, a1);
  scl3(halfaxis, axis, hl);
  const int axisdir = (halfaxis[0] > 0) + 2*(halfaxis[1] > 0) + 4*(halfaxis[2] > 0);
  double bestdist = margin + 2*(size1[0] + hl + size2[0] + size2[1] + size2[2]);
  double bestseg = 0, bestbox = 0, secondpos = -4;
  int cltype = -4, clface = -1, clcorner = 0, cledge = 0;

  /* a segment end against a face: the end clamped onto the box along at most one axis */
  for (int e = -1; e <= 1; e += 2) {
    double p[3], q[3];
    int nclamp = 0, face = -1;
    for (int k = 0; k < 3; k++) {
      p[k] = pos[k] + halfaxis[k]*e;
      q[k] = p[k];
      if (p[k] < -size2[k]) {
        nclamp++;
        face = k;
        p[k] = -size2[k];
      } else if (p[k] > size2[k]) {
        nclamp++;
        face = k;
        p[k] = size2[k];
      }
    }
    if (nclamp > 1) continue;
    for (int k = 0; k < 3; k++) p[k] -= q[k];
    const double dist = dot3(p, p);
    if (dist < bestdist) {
      bestdist = dist;
      bestseg = e;
      cltype = -2 + e;
      clface = face;
    }
  }

  /* the segment against each edge: closest points of two segments, clamped */
  for (int j = 0; j < 3; j++) {
    for (int i = 0; i < 8; i++) {
      if (i & (1 << j)) continue;
      double corner[3] = {((i & 1) ? 1 : -1)*size2[0], ((i & 2) ? 1 : -1)*size2[1],
                          ((i & 4) ? 1 : -1)*size2[2]};
      corner[j] = 0;
      double dif[3];
      sub3(dif, corner, pos);
      const double ma = size2[j]*size2[j], mb = -size2[j]*halfaxis[j], mc = size1[1]*size1[1];
      const double u = -size2[j]*dif[j], v = dot3(halfaxis, dif);
      const double det = ma*mc - mb*mb;
      if (fabs(det) < MINVAL) continue;
      const double idet = 1/det;
      double x1 = (mc*u - mb*v)*idet, x2 = (ma*v - mb*u)*idet;
      int s1 = 1, s2 = 1;
      if (x1 > 1) {
        x1 = 1;
        s1 = 2;
        x2 = (v - mb)*(1/mc);
      } else if (x1 < -1) {
        x1 = -1;
        s1 = 0;
        x2 = (v + mb)*(1/mc);
      }
      if (x2 > 1 || x2 < -1) {
        const int hi = x2 > 1;
        x2 = hi ? 1 : -1;
        s2 = hi ? 2 : 0;
        x1 = (hi ? u - mb : u + mb)*(1/ma);
        if (x1 > 1) {
          x1 = 1;
          s1 = 2;
        } else if (x1 < -1) {
          x1 = -1;
          s1 = 0;
        }
      }
      sub3(dif, corner, pos);
      addToScl3(dif, halfaxis, -x2);
      dif[j] += size2[j]*x1;
      const double d2 = dot3(dif, dif);
      const int t = s1*3 + s2;
      if (d2 < bestdist - MINVAL) {
        bestdist = d2;
        bestseg = x2;
        bestbox = x1;
        clcorner = i + (1 << j)*(t / 6);
        cledge = j;
        cltype = t;
      }
    }
  }
  if (cltype == -4) return 0;

  /* the second point along the segment (:392-559) */
  double mul = 0, e1, e2;
  if (cltype >= 0 && cltype / 3 != 1) {           /* a box corner is closest */
    int c1 = axisdir ^ clcorner, ax = 0, ax1 = 0, ax2 = 0;
    if (c1 != 0 && c1 != 7) {                     /* not pointing at or away from it */
      double de, dp;
      if (c1 == 1 || c1 == 2 || c1 == 4) {
        mul = 1;
        de = 1 - bestseg;
        dp = 1 + bestseg;
      } else {
        mul = -1;
        c1 = 7 - c1;
        dp = 1 - bestseg;
        de = 1 + bestseg;
      }
      if (c1 == 1) { ax = 0; ax1 = 1; ax2 = 2; }
      if (c1 == 2) { ax = 1; ax1 = 2; ax2 = 0; }
      if (c1 == 4) { ax = 2; ax1 = 0; ax2 = 1; }
      if (axis[ax]*axis[ax] > 0.5) {              /* along the box edge */
        secondpos = de;
        e1 = 2*size2[ax]/fabs(halfaxis[ax]);
        if (e1 < secondpos) secondpos = e1;
        secondpos *= mul;
      } else {                                    /* along a box face */
        secondpos = dp;
        e1 = 2*size2[ax1]/fabs(halfaxis[ax1]);
        if (e1 < secondpos) secondpos = e1;
        e1 = 2*size2[ax2]/fabs(halfaxis[ax2]);
        if (e1 < secondpos) secondpos = e1;
        secondpos *= -mul;
      }
    }
  } else if (cltype >= 0) {                       /* the middle of a box edge is closest */
    const int c1 = (axisdir ^ clcorner) & (7 - (1 << cledge));
    if (c1 == 1 || c1 == 2 || c1 == 4) {         /* crossing the edge, not a T */
      int ax = cledge, ax1 = (cledge + 1) % 3, ax2 = (cledge + 2) % 3;
      if (fabs(axis[ax1]) > fabs(axis[ax2])) ax1 = ax2;
      ax2 = 3 - ax - ax1;
      if (c1 & (1 << ax2)) {
        mul = 1;
        secondpos = 1 - bestseg;
      } else {
        mul = -1;
        secondpos = 1 + bestseg;
      }
      e1 = 2*size2[ax2]/fabs(halfaxis[ax2]);
      if (e1 < secondpos) secondpos = e1;
      e2 = (((axisdir & (1 << ax)) != 0) == ((c1 & (1 << ax2)) != 0)) ? 1 - bestbox : 1 + bestbox;
      e1 = size2[ax]*e2/fabs(halfaxis[ax]);
      if (e1 < secondpos) secondpos = e1;
      secondpos *= mul;
    }
  } else if (clface != -1) {                      /* an end against a face, outside the box */
    mul = cltype == -3 ? 1 : -1;
    secondpos = 2;
    double p[3];
    for (int k = 0; k < 3; k++) p[k] = pos[k] + halfaxis[k]*-mul;
    for (int k = 0; k < 3; k++) {
      if (k == clface) continue;
      e1 = (size2[k] - p[k]) / halfaxis[k] * mul;
      if (e1 > 0 && e1 < secondpos) secondpos = e1;
      e1 = (-size2[k] - p[k]) / halfaxis[k] * mul;
      if (e1 > 0 && e1 < secondpos) secondpos = e1;
    }
    secondpos *= mul;
  }

  /* spheres of the capsule's radius at the two points, collided with the box */
  double sp[3], w[3];
  for (int k = 0; k < 3; k++) sp[k] = pos[k] + halfaxis[k]*bestseg;
  mulMatVec3(w, mat2, sp);
  addTo3(w, pos2);
  int n = rawSphereBox(c, margin, w, size1[0], pos2, mat2, size2);
  if (secondpos > -3) {
    for (int k = 0; k < 3; k++) sp[k] = pos[k] + halfaxis[k]*(secondpos + bestseg);
    mulMatVec3(w, mat2, sp);
    addTo3(w, pos2);
    // appended by value (a store through c + n would keep c in private memory)
    RawContact t;
    if (rawSphereBox(&t, margin, w, size1[0], pos2, mat2, size2)) putRaw(c, n++, t);
  }
  return n;
}

// mjraw_CapsuleCapsule
template <class P1, class M1, class P2, class M2>
MJH_HD int colCapsuleCapsule(RawContact* c, double margin, P1 pos1, M1 mat1,
                             const double* size1, P2 pos2, M2 mat2, const double* size2) {
  double axis1[3] = {mat1[2]*size1[1], mat1[5]*size1[1], mat1[8]*size1[1]};
  double axis2[3] = {mat2[2]*size2[1], mat2[5]*size2[1], mat2[8]*size2[1]};
  double dif[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
  double ma = dot3(axis1, axis1);
  double mb = -dot3(axis1, axis2);
  double mc = dot3(axis2, axis2);
  double u = -dot3(axis1, dif);
  double v = dot3(axis2, dif);
  double det = ma*mc - mb*mb;
  double vec1[3], vec2[3];
  if (fabs(det) >= MINVAL) {
    double x1 = (mc*u - mb*v) / det;
    double x2 = (ma*v - mb*u) / det;
    if (x1 > 1) {
      x1 = 1;
      x2 = (v - mb) / mc;
    } else if (x1 < -1) {
      x1 = -1;
      x2 = (v + mb) / mc;
    }
    if (x2 > 1) {
      x2 = 1;
      x1 = clip((u - mb) / ma, -1, 1);
    } else if (x2 < -1) {
      x2 = -1;
      x1 = clip((u + mb) / ma, -1, 1);
    }
    scl3(vec1, axis1, x1);
    addTo3(vec1, pos1);
    scl3(vec2, axis2, x2);
    addTo3(vec2, pos2);
    return rawSphereSphere(c, margin, vec1, mat1, size1[0], vec2, mat2, size2[0]);
  }
  // parallel axes: up to four end-point tests, at most two contacts (each appended to the
  // next free slot of c; the count before an append is 0 or 1)
  RawContact t;
  int n = 0;
  add3(vec1, pos1, axis1);
  double x2 = clip((v - mb) / mc, -1, 1);
  scl3(vec2, axis2, x2);
  addTo3(vec2, pos2);
  if (rawSphereSphere(&t, margin, vec1, mat1, size1[0], vec2, mat2, size2[0])) putRaw(c, n++, t);
  sub3(vec1, pos1, axis1);
  x2 = clip((v + mb) / mc, -1, 1);
  scl3(vec2, axis2, x2);
  addTo3(vec2, pos2);
  if (rawSphereSphere(&t, margin, vec1, mat1, size1[0], vec2, mat2, size2[0])) putRaw(c, n++, t);
  if (n >= 2) return n;
  add3(vec2, pos2, axis2);
  double x1 = clip((u - mb) / ma, -1, 1);
  scl3(vec1, axis1, x1);
  addTo3(vec1, pos1);
  if (rawSphereSphere(&t, margin, vec1, mat1, size1[0], vec2, mat2, size2[0])) putRaw(c, n++, t);
  if (n >= 2) return n;
  sub3(vec2, pos2, axis2);
  x1 = clip((u + mb) / ma, -1, 1);
  scl3(vec1, axis1, x1);
  addTo3(vec1, pos1);
  if (rawSphereSphere(&t, margin, vec1, mat1, size1[0], vec2, mat2, size2[0])) putRaw(c, n++, t);
  return n;
}

// engine_util_spatial.c mju_makeFrame
MJH_HD void makeFrame(double* frame) {
  double tmp[3];
  normalize3(frame);
  if (sqrt(frame[3]*frame[3] + frame[4]*frame[4] + frame[5]*frame[5]) < 0.5) {
    zero3(frame + 3);
    if (frame[1] < 0.5 && frame[1] > -0.5) frame[4] = 1;
    else frame[5] = 1;
  }
  scl3(tmp, frame, dot3(frame, frame + 3));
  sub3(frame + 3, frame + 3, tmp);
  normalize3(frame + 3);
  cross(frame + 6, frame, frame + 3);
}

// mj_contactParam (engine_collision_driver.c:1289-1384), geom : geom
MJH_HD void contactParam(const mjhipModel& m, int g1, int g2, int* condim, double* gap,
                         double* solref, double* solimp, double* friction) {
  double fri[3];
  int p1 = m.geom_priority[g1], p2 = m.geom_priority[g2];
  *gap = m.geom_gap[g1] > m.geom_gap[g2] ? m.geom_gap[g1] : m.geom_gap[g2];
  if (p1 != p2) {
    int g = p1 > p2 ? g1 : g2;
    *condim = m.geom_condim[g];
    for (int i = 0; i < 2; i++) solref[i] = m.geom_solref[2*g+i];
    for (int i = 0; i < 5; i++) solimp[i] = m.geom_solimp[5*g+i];
    for (int i = 0; i < 3; i++) fri[i] = m.geom_friction[3*g+i];
  } else {
    *condim = m.geom_condim[g1] > m.geom_condim[g2] ? m.geom_condim[g1] : m.geom_condim[g2];
    double s1 = m.geom_solmix[g1], s2 = m.geom_solmix[g2], mix;
    if (s1 >= MINVAL && s2 >= MINVAL) mix = s1 / (s1 + s2);
    else if (s1 < MINVAL && s2 < MINVAL) mix = 0.5;
    else if (s1 < MINVAL) mix = 0.0;
    else mix = 1.0;
    const double *r1 = m.geom_solref + 2*g1, *r2 = m.geom_solref + 2*g2;
    if (r1[0] > 0 && r2[0] > 0) {
      for (int i = 0; i < 2; i++) solref[i] = mix*r1[i] + (1-mix)*r2[i];
    } else {
      for (int i = 0; i < 2; i++) solref[i] = r1[i] < r2[i] ? r1[i] : r2[i];
    }
    for (int i = 0; i < 5; i++) solimp[i] = mix*m.geom_solimp[5*g1+i] + (1-mix)*m.geom_solimp[5*g2+i];
    for (int i = 0; i < 3; i++) {
      double a = m.geom_friction[3*g1+i], b = m.geom_friction[3*g2+i];
      fri[i] = a > b ? a : b;
    }
  }
  friction[0] = fri[0];
  friction[1] = fri[0];
  friction[2] = fri[1];
  friction[3] = fri[2];
  friction[4] = fri[2];
}

// mj_filterSphere: 1 = the bounding spheres (or the plane distance) rule the pair out
template <int S>
MJH_HD int filterSphere(const mjhipModel& m, const Lane<S>& d, int g1, int g2, double margin) {
  SP<S> p1 = d.gxpos + 3*g1, p2 = d.gxpos + 3*g2;
  double rb1 = m.geom_rbound[g1], rb2 = m.geom_rbound[g2];
  if (rb1 > 0 && rb2 > 0) {
    double dif[3] = {p1[0]-p2[0], p1[1]-p2[1], p1[2]-p2[2]};
    double bound = rb1 + rb2 + margin;
    return dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2] > bound*bound;
  }
  for (int side = 0; side < 2; side++) {
    int gp = side ? g2 : g1, go = side ? g1 : g2;
    if (m.geom_type[gp] == mjhipGEOM_PLANE && m.geom_rbound[go] > 0) {
      SP<S> mat = d.geom_xmat + 9*gp;
      double norm[3] = {mat[2], mat[5], mat[8]}, dif[3];
      sub3(dif, d.gxpos + 3*go, d.gxpos + 3*gp);
      if (dot3(dif, norm) > margin + m.geom_rbound[go]) return 1;
    }
  }
  return 0;
}

//---------------------------------- box : box (engine_collision_box.c:607-1343) --------------
// Every contact of mjc_BoxBox is final when it is made, so the restatement hands each one
// to emit(RawContact) in the reference's order instead of collecting them in an array.
MJH_HD void bbFaceFrame(int f, double rotmore[9], int idx[3], double sg[3]) {
  for (int k = 0; k < 9; k++) rotmore[k] = 0;
  idx[0] = 0; idx[1] = 1; idx[2] = 2;
  sg[0] = sg[1] = sg[2] = 1;
  switch (f) {
  case 0: rotmore[2] = -1; rotmore[4] = 1; rotmore[6] = 1; idx[0] = 2; sg[0] = -1; idx[2] = 0; break;
  case 1: rotmore[0] = 1; rotmore[5] = -1; rotmore[7] = 1; idx[1] = 2; sg[1] = -1; idx[2] = 1; break;
  case 2: rotmore[0] = 1; rotmore[4] = 1; rotmore[8] = 1; break;
  case 3: rotmore[2] = 1; rotmore[4] = 1; rotmore[6] = -1; idx[0] = 2; idx[2] = 0; sg[2] = -1; break;
  case 4: rotmore[0] = 1; rotmore[5] = 1; rotmore[7] = -1; idx[1] = 2; idx[2] = 1; sg[2] = -1; break;
  default: rotmore[0] = -1; rotmore[4] = 1; rotmore[8] = -1; sg[0] = -1; sg[2] = -1; break;
  }
}
MJH_HD void bbMulMatTMat3(double r[9], const double a[9], const double b[9]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r[3*i+j] = a[i]*b[j] + a[3+i]*b[3+j] + a[6+i]*b[6+j];
}
MJH_HD void bbMulMatMatT3(double r[9], const double a[9], const double b[9]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r[3*i+j] = a[3*i]*b[3*j] + a[3*i+1]*b[3*j+1] + a[3*i+2]*b[3*j+2];
}

template <class F>
MJH_HD void colBoxBox(double margin, const double pos1[3], const double mat1[9],
                      const double size1[3], const double pos2[3], const double mat2[9],
                      const double size2[3], F&& emit) {
  double pos12[3], pos21[3], rot[9], rott[9], rotabs[9], rottabs[9], tmp1[3], tmp2[3];
  double plen1[3], plen2[3], rotmore[9], p[3], r[9], s[3], ss[3], rt[9], sg[3];
  double clnorm[3] = {0, 0, 0}, rnorm[3];
  int idx[3];
  int code = -1, cle1 = 0, cle2 = 0, in = 0;
  const double margin2 = margin*margin;
  sub3(tmp1, pos2, pos1);
  mulMatTVec3(pos21, mat1, tmp1);
  sub3(tmp1, pos1, pos2);
  mulMatTVec3(pos12, mat2, tmp1);
  bbMulMatTMat3(rot, mat1, mat2);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) rott[3*j+i] = rot[3*i+j];
  for (int i = 0; i < 9; i++) rotabs[i] = fabs(rot[i]);
  for (int i = 0; i < 9; i++) rottabs[i] = fabs(rott[i]);
  mulMatVec3(plen2, rotabs, size2);
  mulMatTVec3(plen1, rotabs, size1);
  // separating axes: the six face normals
  double penetration = margin;
  for (int i = 0; i < 3; i++) penetration += size1[i]*3 + size2[i]*3;
  for (int i = 0; i < 3; i++) {
    const double c1 = -fabs(pos21[i]) + size1[i] + plen2[i];
    const double c2 = -fabs(pos12[i]) + size2[i] + plen1[i];
    if (c1 < -margin || c2 < -margin) return;
    if (c1 < penetration) { penetration = c1; code = i + 3*(pos21[i] < 0); }
    if (c2 < penetration) { penetration = c2; code = i + 3*(pos12[i] < 0) + 6; }
  }
  // the nine edge-edge cross products, in box 1's frame
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) {
      tmp2[0] = tmp2[1] = tmp2[2] = 0;
      if (i == 0) { tmp2[1] = -rott[3*j+2]; tmp2[2] = rott[3*j+1]; }
      else if (i == 1) { tmp2[0] = rott[3*j+2]; tmp2[2] = -rott[3*j]; }
      else { tmp2[0] = -rott[3*j+1]; tmp2[1] = rott[3*j]; }
      const double c1 = normalize3(tmp2);
      if (c1 < MINVAL) continue;
      const double c2 = dot3(pos21, tmp2);
      double c3 = 0;
      for (int k = 0; k < 3; k++) if (k != i) c3 += size1[k]*fabs(tmp2[k]);
      for (int k = 0; k < 3; k++) if (k != j) c3 += size2[k]*rotabs[3*i + 3 - k - j] / c1;
      c3 -= fabs(c2);
      if (c3 < -margin) return;
      if (c3 < penetration*(1 - 1e-12)) {
        penetration = c3;
        cle1 = 0;
        for (int k = 0; k < 3; k++) if (k != i && ((tmp2[k] > 0) ^ (c2 < 0))) cle1 += 1 << k;
        cle2 = 0;
        for (int k = 0; k < 3; k++) {
          if (k != j && ((rot[3*i + 3 - k - j] > 0) ^ (c2 < 0) ^ ((k - j + 3) % 3 == 1))) {
            cle2 += 1 << k;
          }
        }
        code = 12 + 3*i + j;
        copy3(clnorm, tmp2);
        in = c2 < 0;
      }
    }
  }
  if (code == -1) return;
  RawContact t;
  for (int k = 3; k < 9; k++) t.frame[k] = 0;

  if (code < 12) {
    // ---- a face of one box against the other box
    const int q1 = code % 6, q2 = code / 6;
    bbFaceFrame(q1, rotmore, idx, sg);
    if (q2) {
      bbMulMatMatT3(r, rotmore, rot);
      for (int k = 0; k < 3; k++) { p[k] = pos12[idx[k]]*sg[k]; tmp1[k] = size2[idx[k]]*sg[k]; }
      copy3(s, size1);
    } else {
      for (int k = 0; k < 3; k++) scl3(r + 3*k, rot + 3*idx[k], sg[k]);
      for (int k = 0; k < 3; k++) { p[k] = pos21[idx[k]]*sg[k]; tmp1[k] = size1[idx[k]]*sg[k]; }
      copy3(s, size2);
    }
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) rt[3*j+i] = r[3*i+j];
    for (int i = 0; i < 3; i++) ss[i] = fabs(tmp1[i]);
    const double lx = ss[0], ly = ss[1], hz = ss[2];
    p[2] -= hz;
    double pts[6][3], lines[4][6];
    copy3(pts[0], p);
    int clcorner = 0;
    for (int i = 0; i < 3; i++) if (r[6+i] < 0) clcorner += 1 << i;
    addToScl3(pts[0], rt, s[0]*((clcorner & 1) ? 1 : -1));
    addToScl3(pts[0], rt + 3, s[1]*((clcorner & 2) ? 1 : -1));
    addToScl3(pts[0], rt + 6, s[2]*((clcorner & 4) ? 1 : -1));
    int m = 1;
    for (int i = 0; i < 3; i++) {
      if (fabs(r[6+i]) < 0.5) {
        scl3(m == 1 ? pts[1] : pts[2], rt + 3*i, s[i]*((clcorner & (1 << i)) ? -2 : 2));
        m++;
      }
    }
    add3(pts[3], pts[0], pts[1]);
    add3(pts[4], pts[0], pts[2]);
    add3(pts[5], pts[3], pts[2]);
    int k = 0;
    if (m > 1) { copy3(lines[0], pts[0]); copy3(lines[0] + 3, pts[1]); k = 1; }
    if (m > 2) {
      copy3(lines[1], pts[0]); copy3(lines[1] + 3, pts[2]);
      copy3(lines[2], pts[3]); copy3(lines[2] + 3, pts[2]);
      copy3(lines[3], pts[4]); copy3(lines[3] + 3, pts[1]);
      k = 4;
    }
    // the contact frame: box q2's face normal, mapped back to the global frame
    double rg[9], pg[3];
    bbMulMatMatT3(rg, q2 ? mat2 : mat1, rotmore);
    copy3(pg, q2 ? pos2 : pos1);
    const double f = q2 ? -1 : 1;
    t.frame[0] = f*rg[2]; t.frame[1] = f*rg[5]; t.frame[2] = f*rg[8];
    auto put = [&](const double pt[3]) MJH_LAMBDA_INLINE {
      if (pt[2] > margin) return;              // the reference's depth filter
      double q[3] = {pt[0], pt[1], pt[2]*0.5};
      t.dist = q[2];                            // half the face depth, as the reference
      q[2] += hz;
      double w[3];
      mulMatVec3(w, rg, q);
      add3(t.pos, w, pg);
      emit(t);
    };
    for (int i = 0; i < k; i++) {             // incident edges against the face's rectangle
      for (int q = 0; q < 2; q++) {
        const double a = lines[i][q], b = lines[i][3+q], cc = lines[i][1-q], dd = lines[i][4-q];
        if (fabs(b) > MINVAL) {
          for (int j = -1; j <= 1; j += 2) {
            const double l = ss[q]*j;
            const double c1 = (l - a)*(1/b);
            if (c1 < 0 || c1 > 1) continue;
            const double c2 = cc + dd*c1;
            if (fabs(c2) > ss[1-q]) continue;
            double pt[3];
            copy3(pt, lines[i]);
            addToScl3(pt, lines[i] + 3, c1);
            put(pt);
          }
        }
      }
    }
    const double a = pts[1][0], b = pts[2][0], cc = pts[1][1], dd = pts[2][1];
    const double c1 = a*dd - b*cc;
    if (m > 2) {                              // face corners inside the incident face
      for (int i = 0; i < 4; i++) {
        const double llx = i/2 ? lx : -lx, lly = i % 2 ? ly : -ly;
        const double x = llx - pts[0][0], y = lly - pts[0][1];
        const double u = (x*dd - y*b)*(1/c1), v = (y*a - x*cc)*(1/c1);
        if (u <= 0 || v <= 0 || u >= 1 || v >= 1) continue;
        const double pt[3] = {llx, lly, pts[0][2] + u*pts[1][2] + v*pts[2][2]};
        put(pt);
      }
    }
    for (int i = 0; i < (1 << (m - 1)); i++) {  // incident corners inside the face
      const double* q = pts[i == 0 ? 0 : i + 2];
      if (i && (q[0] <= -lx || q[0] >= lx)) continue;
      if (i && (q[1] <= -ly || q[1] >= ly)) continue;
      put(q);
    }
    return;
  }

  // ---- edge against edge
  code -= 12;
  const int q1 = code / 3, q2 = code % 3;
  int ax1 = q2 == 0 ? 1 : (q2 == 1 ? 0 : 1), ax2 = q2 == 2 ? 0 : 2;
  int pax1 = q1 == 0 ? 1 : (q1 == 1 ? 0 : 1), pax2 = q1 == 2 ? 0 : 2;
  if (rotabs[3*q1 + ax1] < rotabs[3*q1 + ax2]) { ax1 = ax2; ax2 = 3 - q2 - ax1; }
  if (rottabs[3*q2 + pax1] < rottabs[3*q2 + pax2]) { pax1 = pax2; pax2 = 3 - q1 - pax1; }
  const int clface = (cle1 & (1 << pax2)) ? pax2 : pax2 + 3;
  bbFaceFrame(clface, rotmore, idx, sg);
  for (int k = 0; k < 3; k++) { p[k] = pos21[idx[k]]*sg[k]; rnorm[k] = clnorm[idx[k]]*sg[k]; }
  for (int k = 0; k < 3; k++) scl3(r + 3*k, rot + 3*idx[k], sg[k]);
  mulMatTVec3(tmp1, rotmore, size1);
  for (int i = 0; i < 3; i++) s[i] = fabs(tmp1[i]);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) rt[3*j+i] = r[3*i+j];
  const double lx = s[0], ly = s[1], hz = s[2];
  p[2] -= hz;
  double pu[4][3], ppts2[4][2], axi[3][3], pts[3][3], lines[4][6], linesu[4][6];
  for (int e = 0; e < 2; e++) {            // the incident edge's end points, and the parallel edge's
    double* p0 = pu[2*e];
    copy3(p0, p);
    addToScl3(p0, rt + 3*ax1, size2[ax1]*(((cle2 & (1 << ax1)) ? 1 : -1)*(e ? -1 : 1)));
    addToScl3(p0, rt + 3*ax2, size2[ax2]*((cle2 & (1 << ax2)) ? 1 : -1));
    copy3(pu[2*e + 1], p0);
    addToScl3(p0, rt + 3*q2, size2[q2]);
    addToScl3(pu[2*e + 1], rt + 3*q2, -size2[q2]);
  }
  copy3(axi[0], pu[0]);
  sub3(axi[1], pu[1], pu[0]);
  sub3(axi[2], pu[2], pu[0]);
  if (fabs(rnorm[2]) < MINVAL) return;
  const double innorm = (1/rnorm[2])*(in ? -1 : 1);
  double proj[4][3];
  for (int i = 0; i < 4; i++) {            // project onto the reference face along the normal
    const double c1 = -pu[i][2]*(1/rnorm[2]);
    copy3(proj[i], pu[i]);
    addToScl3(proj[i], rnorm, c1);
    ppts2[i][0] = proj[i][0];
    ppts2[i][1] = proj[i][1];
  }
  copy3(pts[0], proj[0]);
  sub3(pts[1], proj[1], proj[0]);
  sub3(pts[2], proj[2], proj[0]);
  copy3(lines[0], pts[0]); copy3(lines[0] + 3, pts[1]);
  copy3(linesu[0], axi[0]); copy3(linesu[0] + 3, axi[1]);
  copy3(lines[1], pts[0]); copy3(lines[1] + 3, pts[2]);
  copy3(linesu[1], axi[0]); copy3(linesu[1] + 3, axi[2]);
  add3(lines[2], pts[0], pts[1]); copy3(lines[2] + 3, pts[2]);
  add3(linesu[2], axi[0], axi[1]); copy3(linesu[2] + 3, axi[2]);
  add3(lines[3], pts[0], pts[2]); copy3(lines[3] + 3, pts[1]);
  add3(linesu[3], axi[0], axi[2]); copy3(linesu[3] + 3, axi[1]);
  double rg[9];
  bbMulMatMatT3(rg, mat1, rotmore);
  mulMatVec3(tmp1, rg, rnorm);
  scl3(t.frame, tmp1, in ? -1 : 1);
  auto put = [&](double pt[3], double depth) MJH_LAMBDA_INLINE {
    t.dist = depth;
    pt[2] += hz;
    double w[3];
    mulMatVec3(w, rg, pt);
    add3(t.pos, w, pos1);
    emit(t);
  };
  int n = 0;
  for (int i = 0; i < 4; i++) {            // quadrilateral edges against the face rectangle
    for (int q = 0; q < 2; q++) {
      const double a = lines[i][q], b = lines[i][3+q], cc = lines[i][1-q], dd = lines[i][4-q];
      if (fabs(b) > MINVAL) {
        for (int j = -1; j <= 1; j += 2) {
          const double l = s[q]*j;
          const double c1 = (l - a)*(1/b);
          if (c1 < 0 || c1 > 1) continue;
          const double c2 = cc + dd*c1;
          if (fabs(c2) > s[1-q]) continue;
          if ((linesu[i][2] + linesu[i][5]*c1)*innorm > margin) continue;
          double pt[3];
          scl3(pt, linesu[i], 0.5);
          addToScl3(pt, linesu[i] + 3, 0.5*c1);
          pt[q] += 0.5*l;
          pt[1-q] += 0.5*c2;
          put(pt, pt[2]*innorm*2);
          n++;
        }
      }
    }
  }
  const int nl = n;
  const double a = pts[1][0], b = pts[2][0], cc = pts[1][1], dd = pts[2][1];
  double c1 = a*dd - b*cc;
  for (int i = 0; i < 4; i++) {            // face corners against the quadrilateral
    const double llx = i/2 ? lx : -lx, lly = i % 2 ? ly : -ly;
    const double x = llx - pts[0][0], y = lly - pts[0][1];
    double u = (x*dd - y*b)*(1/c1), v = (y*a - x*cc)*(1/c1);
    if (nl == 0) {
      if ((u < 0 || u > 1) && (v < 0 || v > 1)) continue;
    } else if (u < 0 || u > 1 || v < 0 || v > 1) {
      continue;
    }
    u = u < 0 ? 0 : (u > 1 ? 1 : u);
    v = v < 0 ? 0 : (v > 1 ? 1 : v);
    scl3(tmp1, pu[0], 1 - u - v);
    addToScl3(tmp1, pu[1], u);
    addToScl3(tmp1, pu[2], v);
    double pt[3] = {llx, lly, 0};
    sub3(tmp2, pt, tmp1);
    c1 = dot3(tmp2, tmp2);                   // the reference reuses c1 for later corners
    if (tmp1[2] > 0 && c1 > margin2) continue;
    add3(pt, pt, tmp1);
    scl3(pt, pt, 0.5);
    put(pt, sqrt(c1)*(tmp1[2] < 0 ? -1 : 1));
    n++;
  }
  const int nf = n;
  for (int i = 0; i < 4; i++) {            // quadrilateral corners over the face
    const double x = ppts2[i][0], y = ppts2[i][1];
    if (nl == 0) {
      if (nf != 0 && (x < -lx || x > lx) && (y < -ly || y > ly)) continue;
    } else if (x < -lx || x > lx || y < -ly || y > ly) {
      continue;
    }
    double d2 = 0;
    for (int j = 0; j < 2; j++) {
      if (ppts2[i][j] < -s[j]) d2 += (ppts2[i][j] + s[j])*(ppts2[i][j] + s[j]);
      else if (ppts2[i][j] > s[j]) d2 += (ppts2[i][j] - s[j])*(ppts2[i][j] - s[j]);
    }
    d2 += pu[i][2]*innorm*pu[i][2]*innorm;
    if (pu[i][2] > 0 && d2 > margin2) continue;
    double pt[3] = {ppts2[i][0]*0.5, ppts2[i][1]*0.5, 0};
    for (int j = 0; j < 2; j++) {
      if (ppts2[i][j] < -s[j]) pt[j] = -s[j]*0.5;
      else if (ppts2[i][j] > s[j]) pt[j] = s[j]*0.5;
    }
    addToScl3(pt, pu[i], 0.5);
    put(pt, sqrt(d2)*(pu[i][2] < 0 ? -1 : 1));
  }
}

// mju_outsideBox (engine_util_misc.c:911-950): 1 outside the inflated box, -1 inside the
// deflated one, 0 between
MJH_HD int outsideBox(const double point[3], const double pos[3], const double mat[9],
                      const double size[3], double inflate) {
  double vec[3] = {point[0]-pos[0], point[1]-pos[1], point[2]-pos[2]}, v[3];
  mulMatTVec3(v, mat, vec);
  if (v[0] > size[0]*inflate || v[0] < -(size[0]*inflate) || v[1] > size[1]*inflate ||
      v[1] < -(size[1]*inflate) || v[2] > size[2]*inflate || v[2] < -(size[2]*inflate)) {
    return 1;
  }
  const double s0 = size[0]/inflate, s1 = size[1]/inflate, s2 = size[2]/inflate;
  if (v[0] < s0 && v[0] > -s0 && v[1] < s1 && v[1] > -s1 && v[2] < s2 && v[2] > -s2) return -1;
  return 0;
}

// box : box with mj_collideGeoms' clean-up (engine_collision_driver.c:1522-1588): contacts
// outside one box (by 1%) and not inside the other, and earlier copies of a repeated position,
// are dropped. Pass 1 writes each raw contact's position to buf (3 doubles each, at most 24)
// and returns the mask of survivors; pass 2 (boxBoxEmit) regenerates the contacts, which are
// bit-identical, and hands the survivors to store in order.
template <class B>
MJH_HD unsigned boxBoxKeep(double margin, const double pos1[3], const double mat1[9],
                           const double size1[3], const double pos2[3], const double mat2[9],
                           const double size2[3], B buf) {
  const double sz1[3] = {size1[0] + margin, size1[1] + margin, size1[2] + margin};
  const double sz2[3] = {size2[0] + margin, size2[1] + margin, size2[2] + margin};
  unsigned good = 0;
  int num = 0;
  colBoxBox(margin, pos1, mat1, size1, pos2, mat2, size2,
            [&](const RawContact& t) MJH_LAMBDA_INLINE {
    const int o1 = outsideBox(t.pos, pos1, mat1, sz1, 1.01);
    const int o2 = outsideBox(t.pos, pos2, mat2, sz2, 1.01);
    if (!((o1 == 1 && o2 != -1) || (o2 == 1 && o1 != -1))) good |= 1u << num;
    for (int k = 0; k < 3; k++) buf[3*num + k] = t.pos[k];
    num++;
  });
  unsigned keep = good;
  for (int i = 0; i < num - 1; i++) {
    if (!(good >> i & 1)) continue;
    for (int j = i + 1; j < num; j++) {
      if (!(good >> j & 1)) continue;
      if (buf[3*i] == buf[3*j] && buf[3*i+1] == buf[3*j+1] && buf[3*i+2] == buf[3*j+2]) {
        keep &= ~(1u << i);
        break;
      }
    }
  }
  return keep;
}

template <class F>
MJH_HD void boxBoxEmit(double margin, const double pos1[3], const double mat1[9],
                       const double size1[3], const double pos2[3], const double mat2[9],
                       const double size2[3], unsigned keep, F&& store) {
  int num = 0;
  colBoxBox(margin, pos1, mat1, size1, pos2, mat2, size2,
            [&](const RawContact& t) MJH_LAMBDA_INLINE {
    if (keep >> num & 1) store(t);
    num++;
  });
}

//---------------------------------- native convex collision ----------------------------------
// The solver is iterative and stops at ccd_tolerance, so a last-bit change of an operation
// can move its result by that much: everything from here to the end of mjc_ConvexHField is
// compiled without multiply-add contraction, so each operation rounds as in the reference
// (and in the oracle's -ffp-contract=off build); the kernels that feed it their geom frames
// do the same for models with such pairs (codegen.py, exact_fp).
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
// mjc_Convex (engine_collision_convex.c:915-1001, mjENBL_MULTICCD off: one contact) and
// mjc_PlaneConvex (:1045-1080, a geom without mesh data: the ellipsoid) on MuJoCo's native
// GJK/EPA solver mjc_ccd (engine_collision_gjk.c:2215-2343). Everything the solver indexes at
// run time lives in the instance's mirror scratch (d.ccd, d.ccdi, sized by mjh_ccdDoubles /
// mjh_ccdInts), so the contact kernels keep no private arrays:
//   d.ccd   [0, 36)     the GJK simplex, 4 vertices of 9 doubles (Minkowski point, witness on
//                       geom 1, witness on geom 2)
//           [36, 72)    the working simplex of gjkIntersect
//           [72, ...)   the EPA polytope's vertices (5 + ccd_iterations), then per face its
//                       origin projection and distance (4 doubles)
//   d.ccdi  per face vi[3], adj[3] and its slot in the candidate list (-1 none, -2 deleted);
//           the candidate list; the horizon's faces and edges; the horizon search's stack
// The face capacity is 6 ccd_iterations + 6; the reference's is max(6 N, 1000), so a polytope
// that would outgrow ours (never seen) flags the instance MJHIP_INST_UNSUPPORTED instead of
// diverging. The arithmetic is the reference's, operation by operation.

enum { CCD_POINT = 100, CCD_LINE = 101 };   // the shrunken sphere / capsule supports

struct CcdShape {
  int kind, gtype;                          // support in use, the geom's own type
  double pos[3], mat[9], size[3], margin;
  // mesh geoms: the mesh's float vertices and convex-hull graph (null: none), and the warm
  // starts the supports keep between calls (mjCCDObj.vertindex / meshindex)
  const float* vert;
  const int* graph;
  int nvert, vertindex, meshindex;
  int meshid;                               // the mesh (multicontact's polygon data), or -1
  // a height-field prism (mjCCDObj.prism): its three corners' x, y, their top z and the
  // common bottom z (the reference's six vertices share x, y and the bottom z)
  double px[3], py[3], pzt[3], pzb;
};

template <int S>
struct CcdMem {
  SP<S> x;                                  // d.ccd
  SP<S, int> i;                             // d.ccdi
  int nvmax, cap;                           // vertices, faces
  MJH_HD SP<S> sim(int k) const { return x + 9*k; }
  MJH_HD SP<S> wrk(int k) const { return x + 36 + 9*k; }
  MJH_HD SP<S> vtx(int k) const { return x + 72 + 9*k; }
  MJH_HD SP<S> fproj(int f) const { return x + 72 + 9*nvmax + 4*f; }
  // the listed faces' distances, parallel to list(): the closest-face scan reads both
  // arrays in order instead of chasing each entry's face
  MJH_HD SP<S> listd() const { return x + 72 + 9*nvmax + 4*cap; }
  MJH_HD SP<S, int> fint(int f) const { return i + 7*f; }   // vi[0..2], adj[3..5], slot[6]
  MJH_HD SP<S, int> list() const { return i + 7*cap; }
  MJH_HD SP<S, int> hface() const { return i + 8*cap; }
  MJH_HD SP<S, int> hedge() const { return i + 9*cap; }
  MJH_HD SP<S, int> stack() const { return i + 10*cap; }
};

// mulMatTVec3 / localToGlobal (convex.c:122-141)
MJH_HD void ccdToGlobal(double r[3], const double mat[9], const double t[3],
                        const double pos[3]) {
  r[0] = mat[0]*t[0] + mat[1]*t[1] + mat[2]*t[2];
  r[1] = mat[3]*t[0] + mat[4]*t[1] + mat[5]*t[2];
  r[2] = mat[6]*t[0] + mat[7]*t[1] + mat[8]*t[2];
  r[0] += pos[0];
  r[1] += pos[1];
  r[2] += pos[2];
}

// dot product between double and float (convex.c:332-334)
MJH_HD double ccdDot3f(const double a[3], const float* b) {
  return a[0]*(double)b[0] + a[1]*(double)b[1] + a[2]*(double)b[2];
}

// mjc_meshSupport (convex.c:339-382, exhaustive) and mjc_hillclimbSupport (:387-433), as
// mjc_initCCDObj (:735-743) picks them: hill climbing on the hull graph from
// mjMESH_HILLCLIMB_MIN (10) vertices
MJH_HD void ccdMeshSupport(double r[3], CcdShape& s, const double dir[3]) {
  double ld[3], t[3];
  mulMatTVec3(ld, s.mat, dir);
  const float* V = s.vert;
  int imax;
  if (!s.graph || s.nvert < 10) {
    double mx = -3.40282346638528859811704183484516925e+38;   // -FLT_MAX
    imax = 0;
    if (s.vertindex >= 0) {
      imax = s.vertindex;
      mx = ccdDot3f(ld, V + 3*imax);
    }
    for (int i = 0; i < s.nvert; i++) {
      const double vdot = ccdDot3f(ld, V + 3*i);
      if (vdot > mx) {
        mx = vdot;
        imax = i;
      }
    }
    s.vertindex = imax;
  } else {
    const int numvert = s.graph[0];
    const int* edgeadr = s.graph + 2;
    const int* globalid = s.graph + 2 + numvert;
    const int* localid = s.graph + 2 + 2*numvert;
    double mx = -3.40282346638528859811704183484516925e+38;   // -FLT_MAX
    int prev;
    imax = s.meshindex < 0 ? 0 : s.meshindex;
    do {
      prev = imax;
      for (int i = edgeadr[imax]; localid[i] >= 0; i++) {
        const double vdot = ccdDot3f(ld, V + 3*globalid[localid[i]]);
        if (vdot > mx) {
          mx = vdot;
          imax = localid[i];
        }
      }
    } while (imax != prev);
    s.meshindex = imax;
    imax = globalid[imax];
    s.vertindex = imax;
  }
  t[0] = (double)V[3*imax];
  t[1] = (double)V[3*imax + 1];
  t[2] = (double)V[3*imax + 2];
  ccdToGlobal(r, s.mat, t, s.pos);
}

// mjc_prism_support (convex.c:438-455): the best of the three vertices of the half (bottom
// for dir.z < 0, else top), the first on ties, by mju_dot3 of the vertex and dir
MJH_HD void ccdPrismSupport(double r[3], const CcdShape& s, const double dir[3]) {
  const bool bot = dir[2] < 0;
  double z0 = bot ? s.pzb : s.pzt[0];
  double best = s.px[0]*dir[0] + s.py[0]*dir[1] + z0*dir[2];
  double bx = s.px[0], by = s.py[0], bz = z0;
  for (int i = 1; i < 3; i++) {
    const double z = bot ? s.pzb : s.pzt[i];
    const double tmp = s.px[i]*dir[0] + s.py[i]*dir[1] + z*dir[2];
    if (tmp > best) {
      best = tmp;
      bx = s.px[i]; by = s.py[i]; bz = z;
    }
  }
  r[0] = bx; r[1] = by; r[2] = bz;
}

// the native support functions (convex.c:146-327), unit direction
MJH_HD void ccdSupport1(double r[3], CcdShape& s, const double dir[3]) {
  if (s.kind == mjhipGEOM_MESH) {
    ccdMeshSupport(r, s, dir);
    return;
  }
  if (s.kind == mjhipGEOM_HFIELD) {
    ccdPrismSupport(r, s, dir);
    return;
  }
  if (s.kind == CCD_POINT) {
    r[0] = s.pos[0]; r[1] = s.pos[1]; r[2] = s.pos[2];
    return;
  }
  if (s.kind == mjhipGEOM_SPHERE) {
    r[0] = s.size[0]*dir[0] + s.pos[0];
    r[1] = s.size[0]*dir[1] + s.pos[1];
    r[2] = s.size[0]*dir[2] + s.pos[2];
    return;
  }
  double ld[3], t[3];
  mulMatTVec3(ld, s.mat, dir);
  if (s.kind == CCD_LINE) {
    t[0] = 0;
    t[1] = 0;
    t[2] = ld[2] >= 0 ? s.size[1] : -s.size[1];
  } else if (s.kind == mjhipGEOM_CAPSULE) {
    t[0] = ld[0]*s.size[0];
    t[1] = ld[1]*s.size[0];
    t[2] = ld[2]*s.size[0];
    t[2] += ld[2] >= 0 ? s.size[1] : -s.size[1];
  } else if (s.kind == mjhipGEOM_ELLIPSOID) {
    t[0] = ld[0]*s.size[0];
    t[1] = ld[1]*s.size[1];
    t[2] = ld[2]*s.size[2];
    const double nrm = sqrt(t[0]*t[0] + t[1]*t[1] + t[2]*t[2]);
    if (nrm < MINVAL) {
      t[0] = s.size[0]; t[1] = 0; t[2] = 0;
    } else {
      const double inv = 1/nrm;
      t[0] *= inv*s.size[0];
      t[1] *= inv*s.size[1];
      t[2] *= inv*s.size[2];
    }
  } else if (s.kind == mjhipGEOM_CYLINDER) {
    double n = ld[0]*ld[0] + ld[1]*ld[1];
    if (n > MINVAL*MINVAL) {
      n = s.size[0] / sqrt(n);
      t[0] = ld[0]*n;
      t[1] = ld[1]*n;
    } else {
      t[0] = 0; t[1] = 0;
    }
    t[2] = (ld[2] < 0 ? -1.0 : (ld[2] > 0 ? 1.0 : 0.0))*s.size[1];
  } else {                                  // box
    t[0] = (ld[0] >= 0 ? 1.0 : -1.0)*s.size[0];
    t[1] = (ld[1] >= 0 ? 1.0 : -1.0)*s.size[1];
    t[2] = (ld[2] >= 0 ? 1.0 : -1.0)*s.size[2];
  }
  ccdToGlobal(r, s.mat, t, s.pos);
}

// support (gjk.c:277-296) into a 9-double vertex: each shape inflated by half its margin
template <class V>
MJH_HD void ccdSupport(V v, CcdShape& a, CcdShape& b, const double dir[3],
                       const double ndir[3]) {
  double p1[3], p2[3];
  ccdSupport1(p1, a, dir);
  if (a.margin > 0) {
    const double h = 0.5*a.margin;
    p1[0] += dir[0]*h; p1[1] += dir[1]*h; p1[2] += dir[2]*h;
  }
  ccdSupport1(p2, b, ndir);
  if (b.margin > 0) {
    const double h = 0.5*b.margin;
    p2[0] += ndir[0]*h; p2[1] += ndir[1]*h; p2[2] += ndir[2]*h;
  }
  v[0] = p1[0] - p2[0]; v[1] = p1[1] - p2[1]; v[2] = p1[2] - p2[2];
  v[3] = p1[0]; v[4] = p1[1]; v[5] = p1[2];
  v[6] = p2[0]; v[7] = p2[1]; v[8] = p2[2];
}

template <class A, class B> MJH_HD void ccdCopyV(A dst, B src) {
  for (int k = 0; k < 9; k++) dst[k] = src[k];
}

MJH_HD double ccdDet3(const double a[3], const double b[3], const double c[3]) {
  return a[0]*(b[1]*c[2] - b[2]*c[1]) + a[1]*(b[2]*c[0] - b[0]*c[2])
       + a[2]*(b[0]*c[1] - b[1]*c[0]);
}

MJH_HD int ccdSameSign(double a, double b) {
  if (a > 0 && b > 0) return 1;
  if (a < 0 && b < 0) return -1;
  return 0;
}

// projectOriginPlane (gjk.c:482-515): 1 if the plane is degenerate
MJH_HD int ccdProjPlane(double r[3], const double a[3], const double b[3], const double c[3]) {
  double ba[3], ca[3], cb[3], n[3], nv, nn;
  sub3(ba, b, a);
  sub3(ca, c, a);
  sub3(cb, c, b);
  cross(n, cb, ba);
  nv = dot3(n, b);
  nn = dot3(n, n);
  if (nn == 0) return 1;
  if (nv != 0 && nn > MINVAL) {
    scl3(r, n, nv / nn);
    return 0;
  }
  cross(n, ba, ca);
  nv = dot3(n, a);
  nn = dot3(n, n);
  if (nn == 0) return 1;
  if (nv != 0 && nn > MINVAL) {
    scl3(r, n, nv / nn);
    return 0;
  }
  cross(n, ca, cb);
  nv = dot3(n, c);
  nn = dot3(n, n);
  scl3(r, n, nv / nn);
  return 0;
}

// S1D (gjk.c:787-814)
MJH_HD void ccdS1D(double lam[2], const double a[3], const double b[3]) {
  double d[3], p[3];
  sub3(d, b, a);
  const double s = -(dot3(b, d) / dot3(d, d));
  p[0] = b[0] + s*d[0];
  p[1] = b[1] + s*d[1];
  p[2] = b[2] + s*d[2];
  double mu = 0, pi = 0, bi = 0, ai = 0;
  for (int i = 0; i < 3; i++) {
    const double t = a[i] - b[i];
    if (fabs(t) >= fabs(mu)) {
      mu = t; pi = p[i]; bi = b[i]; ai = a[i];
    }
  }
  const double c1 = pi - bi, c2 = ai - pi;
  if (ccdSameSign(mu, c1) && ccdSameSign(mu, c2)) {
    lam[0] = c1 / mu;
    lam[1] = c2 / mu;
  } else {
    lam[0] = 0;
    lam[1] = 1;
  }
}

// minors M_14, M_24, M_34 and the two kept axes (gjk.c:667-714, :979-999); returns M_max
MJH_HD double ccdAxes(const double a[3], const double b[3], const double c[3], int* x, int* y) {
  const double M1 = b[1]*c[2] - b[2]*c[1] - a[1]*c[2] + a[2]*c[1] + a[1]*b[2] - a[2]*b[1];
  const double M2 = b[0]*c[2] - b[2]*c[0] - a[0]*c[2] + a[2]*c[0] + a[0]*b[2] - a[2]*b[0];
  const double M3 = b[0]*c[1] - b[1]*c[0] - a[0]*c[1] + a[1]*c[0] + a[0]*b[1] - a[1]*b[0];
  const double m1 = fabs(M1), m2 = fabs(M2), m3 = fabs(M3);
  if (m1 >= m2 && m1 >= m3) { *x = 1; *y = 2; return M1; }
  if (m2 >= m3) { *x = 0; *y = 2; return M2; }
  *x = 0; *y = 1;
  return M3;
}

// signed area cofactor of (p, u, w) in the kept axes (gjk.c:722-731)
MJH_HD double ccdArea(const double p[3], const double u[3], const double w[3], int x, int y) {
  const double px = x == 0 ? p[0] : p[1], py = y == 1 ? p[1] : p[2];
  const double ux = x == 0 ? u[0] : u[1], uy = y == 1 ? u[1] : u[2];
  const double wx = x == 0 ? w[0] : w[1], wy = y == 1 ? w[1] : w[2];
  return px*uy + py*wx + ux*wy - px*wy - py*ux - wx*uy;
}

// sum of c[k]*v_k, left to right (lincomb, gjk.c:453-477), for 2 or 3 points
MJH_HD void ccdComb2(double r[3], const double l[2], const double a[3], const double b[3]) {
  for (int k = 0; k < 3; k++) r[k] = l[0]*a[k] + l[1]*b[k];
}
MJH_HD void ccdComb3(double r[3], const double l[3], const double a[3], const double b[3],
                     const double c[3]) {
  for (int k = 0; k < 3; k++) r[k] = l[0]*a[k] + l[1]*b[k] + l[2]*c[k];
}

// S2D (gjk.c:653-783)
MJH_HD void ccdS2D(double lam[3], const double a[3], const double b[3], const double c[3]) {
  double p[3];
  if (ccdProjPlane(p, a, b, c)) {
    ccdS1D(lam, a, b);
    lam[2] = 0;
    return;
  }
  int x, y;
  const double Mmax = ccdAxes(a, b, c, &x, &y);
  const double C1 = ccdArea(p, b, c, x, y), C2 = ccdArea(p, c, a, x, y),
               C3 = ccdArea(p, a, b, x, y);
  const int k1 = ccdSameSign(Mmax, C1), k2 = ccdSameSign(Mmax, C2), k3 = ccdSameSign(Mmax, C3);
  if (k1 && k2 && k3) {
    lam[0] = C1 / Mmax;
    lam[1] = C2 / Mmax;
    lam[2] = C3 / Mmax;
    return;
  }
  double dmin = mjhipMAXVAL, l[2], q[3], dd;
  if (!k1) {
    ccdS1D(l, b, c);
    ccdComb2(q, l, b, c);
    dd = dot3(q, q);
    lam[0] = 0; lam[1] = l[0]; lam[2] = l[1];
    dmin = dd;
  }
  if (!k2) {
    ccdS1D(l, a, c);
    ccdComb2(q, l, a, c);
    dd = dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = 0; lam[2] = l[1];
      dmin = dd;
    }
  }
  if (!k3) {
    ccdS1D(l, a, b);
    ccdComb2(q, l, a, b);
    dd = dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = l[1]; lam[2] = 0;
    }
  }
}

// S3D (gjk.c:560-649)
MJH_HD void ccdS3D(double lam[4], const double a[3], const double b[3], const double c[3],
                   const double e[3]) {
  const double C1 = -ccdDet3(b, c, e), C2 = ccdDet3(a, c, e), C3 = -ccdDet3(a, b, e),
               C4 = ccdDet3(a, b, c);
  const double det = C1 + C2 + C3 + C4;
  const int k1 = ccdSameSign(det, C1), k2 = ccdSameSign(det, C2), k3 = ccdSameSign(det, C3),
            k4 = ccdSameSign(det, C4);
  if (k1 && k2 && k3 && k4) {
    lam[0] = C1 / det;
    lam[1] = C2 / det;
    lam[2] = C3 / det;
    lam[3] = C4 / det;
    return;
  }
  double dmin = mjhipMAXVAL, l[3], q[3], dd;
  if (!k1) {
    ccdS2D(l, b, c, e);
    ccdComb3(q, l, b, c, e);
    dd = dot3(q, q);
    lam[0] = 0; lam[1] = l[0]; lam[2] = l[1]; lam[3] = l[2];
    dmin = dd;
  }
  if (!k2) {
    ccdS2D(l, a, c, e);
    ccdComb3(q, l, a, c, e);
    dd = dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = 0; lam[2] = l[1]; lam[3] = l[2];
      dmin = dd;
    }
  }
  if (!k3) {
    ccdS2D(l, a, b, e);
    ccdComb3(q, l, a, b, e);
    dd = dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = l[1]; lam[2] = 0; lam[3] = l[2];
      dmin = dd;
    }
  }
  if (!k4) {
    ccdS2D(l, a, b, c);
    ccdComb3(q, l, a, b, c);
    dd = dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = l[1]; lam[2] = l[2]; lam[3] = 0;
    }
  }
}

// the solver state of one mjc_ccd call (mjCCDStatus, gjk.h:70-89: the fields this path uses)
struct CcdState {
  double dist, x1[3], x2[3];
  int nx, iters, nsimplex, kmax, unsupported;
  double tol, cutoff;
};

template <class V> MJH_HD void ccdLoad3(double r[3], V v) { r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; }

// the face of 3 working-simplex vertices: unit normal and signed distance (gjk.c:375-388)
template <int S>
MJH_HD double ccdFaceDist(double n[3], SP<S> a, SP<S> b, SP<S> c) {
  double va[3], vb[3], vc[3], d1[3], d2[3];
  ccdLoad3(va, a); ccdLoad3(vb, b); ccdLoad3(vc, c);
  sub3(d1, vc, va);
  sub3(d2, vb, va);
  cross(n, d1, d2);
  double nn = dot3(n, n);
  if (nn > MINVAL*MINVAL && nn < mjhipMAXVAL*mjhipMAXVAL) {
    nn = 1/sqrt(nn);
    scl3(n, n, nn);
    return dot3(n, va);
  }
  return mjhipMAXVAL;
}

MJH_HD int ccdPick(int o0, int o1, int o2, int o3, int k) {
  return k == 0 ? o0 : (k == 1 ? o1 : (k == 2 ? o2 : o3));
}

// gjkIntersect (gjk.c:393-448): 1 contact, 0 none, -1 inconclusive
template <int S>
MJH_HD int ccdIntersect(CcdState& st, const CcdMem<S>& M, CcdShape& A, CcdShape& B) {
  for (int q = 0; q < 4; q++) ccdCopyV(M.wrk(q), M.sim(q));
  int o0 = 0, o1 = 1, o2 = 2, o3 = 3;
  int k = st.iters;
  for (; k < st.kmax; k++) {
    double n0[3], n1[3], n2[3], n3[3];
    const double d0 = ccdFaceDist<S>(n0, M.wrk(o2), M.wrk(o1), M.wrk(o3));
    const double d1 = ccdFaceDist<S>(n1, M.wrk(o0), M.wrk(o2), M.wrk(o3));
    const double d2 = ccdFaceDist<S>(n2, M.wrk(o1), M.wrk(o0), M.wrk(o3));
    const double d3 = ccdFaceDist<S>(n3, M.wrk(o0), M.wrk(o1), M.wrk(o2));
    if (!d3 || !d2 || !d1 || !d0) {
      st.iters = k;
      return -1;
    }
    const int i = d0 < d1 ? 0 : 1, j = d2 < d3 ? 2 : 3;
    const double di = i == 0 ? d0 : d1, dj = j == 2 ? d2 : d3;
    const int w = di < dj ? i : j;
    const double dw = di < dj ? di : dj;
    if (dw > 0) {
      st.nsimplex = 4;
      for (int q = 0; q < 4; q++) ccdCopyV(M.sim(q), M.wrk(ccdPick(o0, o1, o2, o3, q)));
      st.iters = k;
      return 1;
    }
    double nw[3];
    for (int c = 0; c < 3; c++) nw[c] = w == 0 ? n0[c] : (w == 1 ? n1[c] : (w == 2 ? n2[c] : n3[c]));
    const double nd[3] = {-nw[0], -nw[1], -nw[2]};
    SP<S> vw = M.wrk(ccdPick(o0, o1, o2, o3, w));
    ccdSupport(vw, A, B, nw, nd);
    if (nw[0]*vw[0] + nw[1]*vw[1] + nw[2]*vw[2] < 0) {
      st.nsimplex = 0;
      st.iters = k;
      return 0;
    }
    // swap entries (w + 1) & 3 and (w + 2) & 3 of the order
    const int a = (w + 1) & 3, b = (w + 2) & 3;
    const int oa = ccdPick(o0, o1, o2, o3, a), ob = ccdPick(o0, o1, o2, o3, b);
    o0 = a == 0 ? ob : (b == 0 ? oa : o0);
    o1 = a == 1 ? ob : (b == 1 ? oa : o1);
    o2 = a == 2 ? ob : (b == 2 ? oa : o2);
    o3 = a == 3 ? ob : (b == 3 ? oa : o3);
  }
  st.iters = k;
  return -1;
}

// gjk (gjk.c:163-272)
template <int S>
MJH_HD void ccdGjk(CcdState& st, const CcdMem<S>& M, CcdShape& A, CcdShape& B) {
  const int get_dist = st.cutoff > 0;
  int backup = !get_dist, n = 0, k = 0;
  double x[3], l0 = 1, l1 = 0, l2 = 0, l3 = 0;
  const double cut2 = st.cutoff*st.cutoff;
  // discreteGeoms (gjk.c:150-158)
  const bool dA = A.gtype == mjhipGEOM_BOX || A.gtype == mjhipGEOM_MESH ||
                  A.gtype == mjhipGEOM_HFIELD;
  const bool dB = B.gtype == mjhipGEOM_BOX || B.gtype == mjhipGEOM_MESH ||
                  B.gtype == mjhipGEOM_HFIELD;
  const bool discrete = A.margin == 0 && B.margin == 0 && dA && dB;
  const double eps = discrete ? 0 : st.tol*st.tol;
  sub3(x, st.x1, st.x2);
  for (; k < st.kmax; k++) {
    double dir[3] = {-1, 0, 0}, ndir[3] = {1, 0, 0};     // gjkSupport (:301-323)
    double nn = dot3(x, x);
    if (nn > MINVAL*MINVAL) {
      nn = 1/sqrt(nn);
      scl3(ndir, x, nn);
      scl3(dir, ndir, -1);
    }
    SP<S> vn = M.sim(n);
    ccdSupport(vn, A, B, dir, ndir);
    double sk[3], diff[3];
    ccdLoad3(sk, vn);
    sub3(diff, x, sk);
    if (2*dot3(x, diff) < eps) {
      if (!k) n = 1;
      break;
    }
    if (!get_dist) {
      if (dot3(x, sk) > 0) {
        st.iters = k; st.nsimplex = 0; st.nx = 0; st.dist = mjhipMAXVAL;
        return;
      }
    } else if (st.cutoff < mjhipMAXVAL) {
      const double vs = dot3(x, sk), vv = dot3(x, x);
      if (dot3(x, sk) > 0 && (vs*vs / vv) >= cut2) {
        st.iters = k; st.nsimplex = 0; st.nx = 0; st.dist = mjhipMAXVAL;
        return;
      }
    }
    if (n == 3 && backup) {
      st.iters = k;
      const int r = ccdIntersect(st, M, A, B);
      if (r != -1) {
        st.nx = 0;
        st.dist = r > 0 ? 0 : mjhipMAXVAL;
        return;
      }
      k = st.iters;
      backup = 0;
    }
    // subdistance (:544-556) on the n + 1 simplex vertices
    double s0[3], s1[3], s2[3], s3[3], lam[4] = {0, 0, 0, 0};
    ccdLoad3(s0, M.sim(0));
    if (n + 1 >= 2) ccdLoad3(s1, M.sim(1));
    if (n + 1 >= 3) ccdLoad3(s2, M.sim(2));
    if (n + 1 == 4) ccdLoad3(s3, M.sim(3));
    if (n + 1 == 4) ccdS3D(lam, s0, s1, s2, s3);
    else if (n + 1 == 3) ccdS2D(lam, s0, s1, s2);
    else if (n + 1 == 2) ccdS1D(lam, s0, s1);
    else lam[0] = 1;
    // drop the vertices with zero weight, in order
    const double L[4] = {lam[0], lam[1], lam[2], lam[3]};
    n = 0;
    l0 = 0; l1 = 0; l2 = 0; l3 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (L[i] == 0) continue;
      if (n != i) ccdCopyV(M.sim(n), M.sim(i));
      l0 = n == 0 ? L[i] : l0;
      l1 = n == 1 ? L[i] : l1;
      l2 = n == 2 ? L[i] : l2;
      l3 = n == 3 ? L[i] : l3;
      n++;
    }
    // the next iterate (lincomb of the n kept vertices)
    double nx[3];
    for (int c = 0; c < 3; c++) {
      double s = l0*M.sim(0)[c];
      if (n > 1) s = s + l1*M.sim(1)[c];
      if (n > 2) s = s + l2*M.sim(2)[c];
      if (n > 3) s = s + l3*M.sim(3)[c];
      nx[c] = s;
    }
    if (fabs(nx[0] - x[0]) < MINVAL && fabs(nx[1] - x[1]) < MINVAL &&
        fabs(nx[2] - x[2]) < MINVAL) {
      break;
    }
    copy3(x, nx);
    if (n == 4) break;
  }
  // the witness points: lincomb of the kept vertices' witnesses
  for (int c = 0; c < 3; c++) {
    double s1v = l0*M.sim(0)[3 + c], s2v = l0*M.sim(0)[6 + c];
    if (n > 1) { s1v = s1v + l1*M.sim(1)[3 + c]; s2v = s2v + l1*M.sim(1)[6 + c]; }
    if (n > 2) { s1v = s1v + l2*M.sim(2)[3 + c]; s2v = s2v + l2*M.sim(2)[6 + c]; }
    if (n > 3) { s1v = s1v + l3*M.sim(3)[3 + c]; s2v = s2v + l3*M.sim(3)[6 + c]; }
    st.x1[c] = s1v;
    st.x2[c] = s2v;
  }
  st.nx = 1;
  st.iters = k;
  st.nsimplex = n;
  st.dist = sqrt(x[0]*x[0] + x[1]*x[1] + x[2]*x[2]);
}

//------------------------------------- EPA (gjk.c:820-1459) ----------------------------------

// polytope bookkeeping kept in registers
struct CcdPoly {
  int nvtx, nface, nlist, nh;
};

template <int S>
MJH_HD int ccdAddVertex(const CcdMem<S>& M, CcdPoly& P, SP<S> v) {
  SP<S> t = M.vtx(P.nvtx);
  for (int k = 3; k < 9; k++) t[k] = v[k];
  t[0] = v[3] - v[6]; t[1] = v[4] - v[7]; t[2] = v[5] - v[8];
  return P.nvtx++;
}

// epaSupport (:328-353)
// (w, when given, receives the vertex's Minkowski point from registers)
template <int S>
MJH_HD int ccdNewVertex(const CcdMem<S>& M, CcdPoly& P, CcdShape& A, CcdShape& B,
                        const double d[3], double dn, double* w = nullptr) {
  double dir[3] = {1, 0, 0}, ndir[3] = {-1, 0, 0};
  if (dn > MINVAL) {
    dir[0] = d[0] / dn;
    dir[1] = d[1] / dn;
    dir[2] = d[2] / dn;
    scl3(ndir, dir, -1);
  }
  double v[9];
  ccdSupport(v, A, B, dir, ndir);
  SP<S> t = M.vtx(P.nvtx);
  for (int k = 0; k < 9; k++) t[k] = v[k];
  if (w) {
    w[0] = v[0]; w[1] = v[1]; w[2] = v[2];
  }
  return P.nvtx++;
}

// attachFace (:1192-1213)
template <int S>
MJH_HD double ccdAttach(const CcdMem<S>& M, CcdPoly& P, int a, int b, int c, int j1, int j2,
                        int j3) {
  const int f = P.nface++;
  SP<S, int> fi = M.fint(f);
  fi[0] = a; fi[1] = b; fi[2] = c; fi[3] = j1; fi[4] = j2; fi[5] = j3;
  double va[3], vb[3], vc[3], pr[3];
  ccdLoad3(va, M.vtx(a)); ccdLoad3(vb, M.vtx(b)); ccdLoad3(vc, M.vtx(c));
  if (ccdProjPlane(pr, vc, vb, va)) return 0;
  SP<S> fp = M.fproj(f);
  fp[0] = pr[0]; fp[1] = pr[1]; fp[2] = pr[2];
  const double dist = sqrt(pr[0]*pr[0] + pr[1]*pr[1] + pr[2]*pr[2]);
  fp[3] = dist;
  fi[6] = -1;
  return dist;
}

template <int S>
MJH_HD void ccdListAll(const CcdMem<S>& M, CcdPoly& P, int n) {
  for (int i = 0; i < n; i++) {
    M.list()[i] = i;
    M.listd()[i] = M.fproj(i)[3];
    M.fint(i)[6] = i;
  }
  P.nlist = n;
}

// replaceSimplex3 (:820-837)
template <int S>
MJH_HD void ccdToTriangle(const CcdMem<S>& M, CcdPoly& P, CcdState& st, int a, int b, int c) {
  st.nsimplex = 3;
  ccdCopyV(M.sim(0), M.vtx(a));
  ccdCopyV(M.sim(1), M.vtx(b));
  ccdCopyV(M.sim(2), M.vtx(c));
  P.nface = 0;
  P.nvtx = 0;
}

// sameSide / testTetra (:842-868)
MJH_HD int ccdSameSide(const double p0[3], const double p1[3], const double p2[3],
                       const double p3[3]) {
  double e1[3], e2[3], e3[3], e4[3], n[3];
  sub3(e1, p1, p0);
  sub3(e2, p2, p0);
  cross(n, e1, e2);
  sub3(e3, p3, p0);
  const double d1 = dot3(n, e3);
  scl3(e4, p0, -1);
  const double d2 = dot3(n, e4);
  return (d1 > 0 && d2 > 0) || (d1 < 0 && d2 < 0);
}

MJH_HD int ccdInTetra(const double a[3], const double b[3], const double c[3],
                      const double d[3]) {
  return ccdSameSide(a, b, c, d) && ccdSameSide(b, c, d, a) && ccdSameSide(c, d, a, b) &&
         ccdSameSide(d, a, b, c);
}

// triAffineCoord / triPointIntersect (:976-1035)
MJH_HD void ccdAffine(double lam[3], const double a[3], const double b[3], const double c[3],
                      const double p[3]) {
  int x, y;
  const double Mmax = ccdAxes(a, b, c, &x, &y);
  lam[0] = ccdArea(p, b, c, x, y) / Mmax;
  lam[1] = ccdArea(p, c, a, x, y) / Mmax;
  lam[2] = ccdArea(p, a, b, x, y) / Mmax;
}

MJH_HD int ccdOnTriangle(const double a[3], const double b[3], const double c[3],
                         const double p[3]) {
  double lam[3], q[3], d[3];
  ccdAffine(lam, a, b, c, p);
  if (lam[0] < 0 || lam[1] < 0 || lam[2] < 0) return 0;
  q[0] = a[0]*lam[0] + b[0]*lam[1] + c[0]*lam[2];
  q[1] = a[1]*lam[0] + b[1]*lam[1] + c[1]*lam[2];
  q[2] = a[2]*lam[0] + b[2]*lam[1] + c[2]*lam[2];
  sub3(d, q, p);
  return sqrt(d[0]*d[0] + d[1]*d[1] + d[2]*d[2]) < MINVAL;
}

// polytope3 (:1040-1117)
template <int S>
MJH_HD int ccdFromTriangle(const CcdMem<S>& M, CcdPoly& P, CcdState& st, CcdShape& A,
                           CcdShape& B) {
  double a[3], b[3], c[3], e1[3], e2[3], n[3], nn[3];
  ccdLoad3(a, M.sim(0)); ccdLoad3(b, M.sim(1)); ccdLoad3(c, M.sim(2));
  sub3(e1, b, a);
  sub3(e2, c, a);
  cross(n, e1, e2);
  const double nrm = sqrt(n[0]*n[0] + n[1]*n[1] + n[2]*n[2]);
  if (nrm < MINVAL) return 4;                           // mjEPA_P3_BAD_NORMAL
  scl3(nn, n, -1);
  const int i1 = ccdAddVertex(M, P, M.sim(0));
  const int i2 = ccdAddVertex(M, P, M.sim(1));
  const int i3 = ccdAddVertex(M, P, M.sim(2));
  const int i5 = ccdNewVertex(M, P, A, B, nn, nrm);
  const int i4 = ccdNewVertex(M, P, A, B, n, nrm);
  double v4[3], v5[3];
  ccdLoad3(v4, M.vtx(i4));
  ccdLoad3(v5, M.vtx(i5));
  if (ccdOnTriangle(a, b, c, v4)) return 5;            // mjEPA_P3_INVALID_V4
  if (ccdOnTriangle(a, b, c, v5)) return 6;            // mjEPA_P3_INVALID_V5
  if (st.dist > 10*MINVAL && !ccdInTetra(a, b, c, v4) && !ccdInTetra(a, b, c, v5)) return 7;
  if (ccdAttach(M, P, i4, i1, i2, 1, 3, 2) < MINVAL) return 8;
  if (ccdAttach(M, P, i4, i3, i1, 2, 4, 0) < MINVAL) return 8;
  if (ccdAttach(M, P, i4, i2, i3, 0, 5, 1) < MINVAL) return 8;
  if (ccdAttach(M, P, i5, i2, i1, 5, 0, 4) < MINVAL) return 8;
  if (ccdAttach(M, P, i5, i1, i3, 3, 1, 5) < MINVAL) return 8;
  if (ccdAttach(M, P, i5, i3, i2, 4, 2, 3) < MINVAL) return 8;   // mjEPA_P3_ORIGIN_ON_FACE
  ccdListAll(M, P, 6);
  return 0;
}

// polytope2 (:892-971)
template <int S>
MJH_HD int ccdFromSegment(const CcdMem<S>& M, CcdPoly& P, CcdState& st, CcdShape& A,
                          CcdShape& B) {
  double a[3], b[3], d[3];
  ccdLoad3(a, M.sim(0)); ccdLoad3(b, M.sim(1));
  sub3(d, b, a);
  double best = mjhipMAXVAL;
  int ix = 0;
  for (int i = 0; i < 3; i++) {
    if (fabs(d[i]) < best) {
      best = fabs(d[i]);
      ix = i;
    }
  }
  double e[3] = {ix == 0 ? 1.0 : 0.0, ix == 1 ? 1.0 : 0.0, ix == 2 ? 1.0 : 0.0};
  double d1[3], d2[3], d3[3], R[9];
  cross(d1, e, d);
  {                                                     // rotmat (:873-887): 120 degrees
    const double n = sqrt(d[0]*d[0] + d[1]*d[1] + d[2]*d[2]);
    const double u1 = d[0] / n, u2 = d[1] / n, u3 = d[2] / n;
    const double sn = 0.86602540378, cs = -0.5;
    R[0] = cs + u1*u1*(1 - cs);
    R[1] = u1*u2*(1 - cs) - u3*sn;
    R[2] = u1*u3*(1 - cs) + u2*sn;
    R[3] = u2*u1*(1 - cs) + u3*sn;
    R[4] = cs + u2*u2*(1 - cs);
    R[5] = u2*u3*(1 - cs) - u1*sn;
    R[6] = u1*u3*(1 - cs) - u2*sn;
    R[7] = u2*u3*(1 - cs) + u1*sn;
    R[8] = cs + u3*u3*(1 - cs);
  }
  mulMatVec3(d2, R, d1);
  mulMatVec3(d3, R, d2);
  const int i1 = ccdAddVertex(M, P, M.sim(0));
  const int i2 = ccdAddVertex(M, P, M.sim(1));
  const int i3 = ccdNewVertex(M, P, A, B, d1, sqrt(d1[0]*d1[0] + d1[1]*d1[1] + d1[2]*d1[2]));
  const int i4 = ccdNewVertex(M, P, A, B, d2, sqrt(d2[0]*d2[0] + d2[1]*d2[1] + d2[2]*d2[2]));
  const int i5 = ccdNewVertex(M, P, A, B, d3, sqrt(d3[0]*d3[0] + d3[1]*d3[1] + d3[2]*d3[2]));
  // the hexahedron's faces (vertices, adjacent faces); a face through the origin makes the
  // simplex that face's triangle
  const int tv[6][3] = {{i1, i3, i4}, {i1, i5, i3}, {i1, i4, i5},
                        {i2, i4, i3}, {i2, i3, i5}, {i2, i5, i4}};
  const int ta[6][3] = {{1, 3, 2}, {2, 4, 0}, {0, 5, 1}, {5, 0, 4}, {3, 1, 5}, {4, 2, 3}};
#pragma unroll
  for (int f = 0; f < 6; f++) {
    if (ccdAttach(M, P, tv[f][0], tv[f][1], tv[f][2], ta[f][0], ta[f][1], ta[f][2]) < MINVAL) {
      ccdToTriangle(M, P, st, tv[f][0], tv[f][1], tv[f][2]);
      return ccdFromTriangle(M, P, st, A, B);
    }
  }
  double v1[3], v2[3], v3[3], v4[3], v5[3];
  ccdLoad3(v1, M.vtx(i1)); ccdLoad3(v2, M.vtx(i2)); ccdLoad3(v3, M.vtx(i3));
  ccdLoad3(v4, M.vtx(i4)); ccdLoad3(v5, M.vtx(i5));
  if (st.dist > 10*MINVAL && !ccdInTetra(v1, v3, v4, v5) && !ccdInTetra(v2, v3, v4, v5)) {
    return 2;                                           // mjEPA_P2_MISSING_ORIGIN
  }
  ccdListAll(M, P, 6);
  return 0;
}

// polytope4 (:1122-1156)
template <int S>
MJH_HD int ccdFromTetra(const CcdMem<S>& M, CcdPoly& P, CcdState& st, CcdShape& A,
                        CcdShape& B) {
  const int i1 = ccdAddVertex(M, P, M.sim(0));
  const int i2 = ccdAddVertex(M, P, M.sim(1));
  const int i3 = ccdAddVertex(M, P, M.sim(2));
  const int i4 = ccdAddVertex(M, P, M.sim(3));
  const int tv[4][3] = {{i1, i2, i3}, {i1, i4, i2}, {i1, i3, i4}, {i4, i3, i2}};
  const int ta[4][3] = {{1, 3, 2}, {2, 3, 0}, {0, 3, 1}, {2, 0, 1}};
#pragma unroll
  for (int f = 0; f < 4; f++) {
    if (ccdAttach(M, P, tv[f][0], tv[f][1], tv[f][2], ta[f][0], ta[f][1], ta[f][2]) < MINVAL) {
      ccdToTriangle(M, P, st, tv[f][0], tv[f][1], tv[f][2]);
      return ccdFromTriangle(M, P, st, A, B);
    }
  }
  double v1[3], v2[3], v3[3], v4[3];
  ccdLoad3(v1, M.vtx(i1)); ccdLoad3(v2, M.vtx(i2)); ccdLoad3(v3, M.vtx(i3));
  ccdLoad3(v4, M.vtx(i4));
  if (!ccdInTetra(v1, v2, v3, v4)) return 9;            // mjEPA_P4_MISSING_ORIGIN
  ccdListAll(M, P, 4);
  return 0;
}

// deleteFace (:1174-1180)
template <int S>
MJH_HD void ccdUnlist(const CcdMem<S>& M, CcdPoly& P, int f) {
  SP<S, int> fi = M.fint(f);
  const int slot = fi[6];
  if (slot >= 0) {
    const int moved = M.list()[--P.nlist];
    const double md = M.listd()[P.nlist];
    M.list()[slot] = moved;
    M.listd()[slot] = md;
    M.fint(moved)[6] = slot;
  }
  fi[6] = -2;
}

template <int S>
MJH_HD int ccdEdgeOf(const CcdMem<S>& M, int f, int v) {
  SP<S, int> fi = M.fint(f);
  if (fi[0] == v) return 0;
  if (fi[1] == v) return 1;
  return 2;
}

// whether face f sees w (horizonRec's test, :1247-1250)
template <int S>
MJH_HD bool ccdSees(const CcdMem<S>& M, int f, const double w[3]) {
  SP<S> fp = M.fproj(f);
  const double d2 = fp[3]*fp[3];
  return fp[0]*w[0] + fp[1]*w[1] + fp[2]*w[2] >= d2;
}

// horizon (:1217-1295): the depth-first search of horizonRec with an explicit stack of
// (face, entry edge, next k); a neighbour that does not see w is a horizon edge, one that
// does is deleted and searched, in the recursion's order. false: more horizon edges than the
// reference's horizon arrays hold, or the stack outgrew the face capacity.
// The polytope lives in memory, where a load issued after a store waits for it: the frame
// being searched stays in registers (only its parents go to the stack), a face's vertices,
// neighbours and projection never change during the search and are loaded with its list
// slot in one batch, so a step of the search costs one memory round trip.
template <int S>
MJH_HD bool ccdHorizon(const CcdMem<S>& M, CcdPoly& P, int f0, const double w[3], int hmax) {
  SP<S, int> stk = M.stack();
  SP<S, int> hf = M.hface(), he = M.hedge();
  // face x: fi[0..6] (vertices, neighbours, list slot) and fp[0..3] (projection)
  auto loadFace = [&](int x, int fi[7], double fp[4]) MJH_LAMBDA_INLINE {
    SP<S, int> F = M.fint(x);
    SP<S> Q = M.fproj(x);
    for (int q = 0; q < 7; q++) fi[q] = F[q];
    for (int q = 0; q < 4; q++) fp[q] = Q[q];
  };
  auto sees = [&](const double fp[4]) MJH_LAMBDA_INLINE {
    return fp[0]*w[0] + fp[1]*w[1] + fp[2]*w[2] >= fp[3]*fp[3];
  };
  auto edgeOf = [&](const int fi[7], int v) MJH_LAMBDA_INLINE {
    return fi[0] == v ? 0 : (fi[1] == v ? 1 : 2);
  };
  // deleteFace with the face's list slot already loaded
  auto unlist = [&](int x, int slot) MJH_LAMBDA_INLINE {
    if (slot >= 0) {
      const int moved = M.list()[--P.nlist];
      const double md = M.listd()[P.nlist];
      M.list()[slot] = moved;
      M.listd()[slot] = md;
      M.fint(moved)[6] = slot;
    }
    M.fint(x)[6] = -2;
  };
  int a0[7];
  double p0[4];
  loadFace(f0, a0, p0);
  unlist(f0, a0[6]);
  for (int k0 = 0; k0 < 3; k0++) {
    const int g = a0[3 + k0];
    int gi[7];
    double gp[4];
    loadFace(g, gi, gp);                   // after the previous searches' deletions
    const int ge = edgeOf(gi, a0[(k0 + 1) % 3]);
    if (k0 > 0 && gi[6] <= -2) continue;
    if (!sees(gp)) {
      if (P.nh >= hmax) return false;
      hf[P.nh] = g; he[P.nh] = ge; P.nh++;
      continue;
    }
    unlist(g, gi[6]);
    int top = 0;                            // frames below the current one on the stack
    int f = g, e = ge, k = 1;
    int fa[7];
    for (int q = 0; q < 7; q++) fa[q] = gi[q];
    while (true) {
      if (k == 3) {
        if (top == 0) break;
        top--;
        SP<S, int> fr = stk + 3*top;
        f = fr[0]; e = fr[1]; k = fr[2];
        SP<S, int> F = M.fint(f);
        for (int q = 0; q < 6; q++) fa[q] = F[q];
        continue;
      }
      const int i = (e + k) % 3;
      k++;
      const int h = fa[3 + i];
      int hi[7];
      double hp[4];
      loadFace(h, hi, hp);
      if (hi[6] > -2) {
        const int hge = edgeOf(hi, fa[(i + 1) % 3]);
        if (sees(hp)) {
          unlist(h, hi[6]);
          if (3*(top + 2) > 3*M.cap) return false;
          SP<S, int> fr = stk + 3*top;      // the parent, resumed at its next k
          fr[0] = f; fr[1] = e; fr[2] = k;
          top++;
          f = h; e = hge; k = 1;
          for (int q = 0; q < 7; q++) fa[q] = hi[q];
        } else {
          if (P.nh >= hmax) return false;
          hf[P.nh] = h; he[P.nh] = hge; P.nh++;
        }
      }
    }
  }
  return true;
}

// epa (:1329-1459) + epaWitness (:1300-1323): the face closest to the origin, or -1
template <int S>
MJH_HD int ccdEpa(CcdState& st, const CcdMem<S>& M, CcdPoly& P, CcdShape& A,
                  CcdShape& B) {
  const double FLTMAX = 3.40282346638528859811704183484516925e+38;   // FLT_MAX
  const int refmax = 6*st.kmax > 1000 ? 6*st.kmax : 1000;            // the reference's faces
  double lower, upper = FLTMAX;
  int f = -1, pf = -1, k;
  P.nh = 0;
  for (k = 0; k < st.kmax; k++) {
    pf = f;
    lower = FLTMAX;
    // the closest listed face, scanned in list order (ties keep the earlier face) over the
    // list and its parallel distances (listd): sixteen entries' loads are issued before
    // their compares, so a scan of n faces waits for n / 16 memory round trips
    int i = 0;
    for (; i + 16 <= P.nlist; i += 16) {
      int g16[16];
      double d16[16];
#pragma unroll
      for (int u = 0; u < 16; u++) {
        g16[u] = M.list()[i + u];
        d16[u] = M.listd()[i + u];
      }
#pragma unroll
      for (int u = 0; u < 16; u++) {
        if (d16[u] < lower) {
          f = g16[u];
          lower = d16[u];
        }
      }
    }
    for (; i < P.nlist; i++) {
      const int g = M.list()[i];
      const double dg = M.listd()[i];
      if (dg < lower) {
        f = g;
        lower = dg;
      }
    }
    if (lower > upper || f < 0) {
      f = pf;
      break;
    }
    if (lower <= 0) break;                              // origin on a face (a warning)
    double fp[3], w[3];
    ccdLoad3(fp, M.fproj(f));
    if (P.nvtx >= M.nvmax) {                            // cannot happen: one per iteration
      st.unsupported = 1;
      return -1;
    }
    const int wi = ccdNewVertex(M, P, A, B, fp, lower, w);
    const double up = (fp[0]*w[0] + fp[1]*w[1] + fp[2]*w[2]) / lower;
    if (up < upper) upper = up;
    if (upper - lower < st.tol) break;
    if (!ccdHorizon(M, P, f, w, 6 + st.kmax)) {
      st.unsupported = 1;
      return -1;
    }
    if (P.nh < 3) {
      f = -1;
      break;
    }
    const int nf = P.nface, ne = P.nh;
    if (ne > refmax - P.nface) break;                   // out of face memory (a warning)
    if (ne > M.cap - P.nface) {                         // ours is smaller: not this engine's
      st.unsupported = 1;
      return -1;
    }
    // the new faces (attachFace per horizon edge, in order), eight edges at a time: what
    // they read (the horizon faces' vertices, the vertices' points) never changes here, so
    // it is loaded before the chunk's stores; a degenerate face ends the search (f = -1,
    // after which the polytope is not read again)
    for (int i0 = 0; i0 < ne && f >= 0; i0 += 8) {
      const int cnt = ne - i0 < 8 ? ne - i0 : 8;
      int hfi[8], he8[8], a8[8], b8[8];
      double va[8][3], vb[8][3];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (u < cnt) {
          hfi[u] = M.hface()[i0 + u];
          he8[u] = M.hedge()[i0 + u];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (u < cnt) {
          SP<S, int> H = M.fint(hfi[u]);
          a8[u] = H[he8[u]];
          b8[u] = H[(he8[u] + 1) % 3];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (u < cnt) {
          ccdLoad3(va[u], M.vtx(a8[u]));
          ccdLoad3(vb[u], M.vtx(b8[u]));
        }
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (u >= cnt) break;
        const int i = i0 + u;
        const int cur = nf + i, prev = i ? cur - 1 : nf + ne - 1, next = nf + (i + 1) % ne;
        M.fint(hfi[u])[3 + he8[u]] = cur;
        // attachFace(wi, b, a, prev, hfi, next) with its vertices from registers
        const int nfc = P.nface++;
        SP<S, int> fi = M.fint(nfc);
        fi[0] = wi; fi[1] = b8[u]; fi[2] = a8[u]; fi[3] = prev; fi[4] = hfi[u]; fi[5] = next;
        double pr[3], dd = 0;
        if (!ccdProjPlane(pr, va[u], vb[u], w)) {
          SP<S> fq = M.fproj(nfc);
          fq[0] = pr[0]; fq[1] = pr[1]; fq[2] = pr[2];
          dd = sqrt(pr[0]*pr[0] + pr[1]*pr[1] + pr[2]*pr[2]);
          fq[3] = dd;
          fi[6] = -1;
        }
        if (dd == 0) {
          f = -1;
          break;
        }
        if (dd >= lower && dd <= upper) {
          const int s = P.nlist++;
          M.list()[s] = nfc;
          M.listd()[s] = dd;
          fi[6] = s;
        }
      }
    }
    P.nh = 0;
    if (!P.nlist || f < 0) break;
  }
  if (f >= 0) {
    SP<S, int> F = M.fint(f);
    double a[3], b[3], c[3], pr[3], lam[3];
    ccdLoad3(a, M.vtx(F[0])); ccdLoad3(b, M.vtx(F[1])); ccdLoad3(c, M.vtx(F[2]));
    ccdLoad3(pr, M.fproj(f));
    ccdAffine(lam, a, b, c, pr);
    SP<S> va = M.vtx(F[0]), vb = M.vtx(F[1]), vc = M.vtx(F[2]);
    for (int i = 0; i < 3; i++) {
      st.x1[i] = va[3 + i]*lam[0] + vb[3 + i]*lam[1] + vc[3 + i]*lam[2];
      st.x2[i] = va[6 + i]*lam[0] + vb[6 + i]*lam[1] + vc[6 + i]*lam[2];
    }
    st.nx = 1;
    st.dist = -M.fproj(f)[3];
  } else {
    st.nx = 0;
    st.dist = 0;
  }
  return f;
}

// obj->center: the geom position (mjc_center convex.c:78-98), or a prism's mean vertex
// (mjc_prism_center :103-110: zero, add the six vertices in order, scale by 1/6)
MJH_HD void ccdCenter(double c[3], const CcdShape& s) {
  if (s.gtype == mjhipGEOM_HFIELD) {
    c[0] = 0; c[1] = 0; c[2] = 0;
    for (int i = 0; i < 3; i++) { c[0] += s.px[i]; c[1] += s.py[i]; c[2] += s.pzb; }
    for (int i = 0; i < 3; i++) { c[0] += s.px[i]; c[1] += s.py[i]; c[2] += s.pzt[i]; }
    scl3(c, c, 1.0/6.0);
  } else {
    copy3(c, s.pos);
  }
}

// ---- multicontact (engine_collision_gjk.c:1460-2193), box pairs: with max_contacts > 1 the
// EPA's final face becomes a contact polygon -- each geom's feature spanned by the face's three
// vertices, the face normals around it, a pair of anti-aligned faces (or an edge perpendicular
// to a face), one face clipped by the other's edge planes. The reference keeps each polytope
// vertex's box corner (Vertex.index1/2, set by mjc_boxSupport's vertindex); here the corner is
// read back from the witness point itself -- the sign pattern of its box-frame coordinates,
// which is the support's `tmp` sign pattern -- so the solver's memory layout is unchanged.
// A mesh vertex is read back by finding the vertex whose global position is the witness point
// bit for bit (the support computed it from that vertex with the same operations); the mesh
// polygons are the compiler's (mjCMesh::MakePolygons, meshes.py). Only k_ccd (mjhip_ccdBatch)
// compiles this in (ccdRun's MULTI), with private arrays sized for polygons of up to
// CCD_MAXFACE vertices and vertices on up to CCD_MAXFACE polygons (the reference's bound is
// mjMAX_POLYVERT = 150; a larger one is refused, MJHIP_ERR_MODEL).
constexpr double CCD_FACE_TOL = 0.99999872;     // mjFACE_TOL (gjk.h:29)
constexpr double CCD_EDGE_TOL = 0.00159999931;  // mjEDGE_TOL (gjk.h:32)
constexpr int CCD_MAXCON = 50;                  // mjMAXCONPAIR: the witness capacity
constexpr int CCD_MAXFACE = 16;                 // polygon vertices / polygons at a vertex
constexpr int CCD_MAXPOLY = 2*CCD_MAXFACE;      // clipped polygon capacity

// the box corner a support point is (mjc_boxSupport's vertindex bits, convex.c:319-323)
MJH_HD int ccdBoxCorner(const CcdShape& s, const double* p) {
  double d[3], l[3];
  sub3(d, p, s.pos);
  mulMatTVec3(l, s.mat, d);
  return (l[0] > 0 ? 1 : 0) | (l[1] > 0 ? 2 : 0) | (l[2] > 0 ? 4 : 0);
}

// area4 (:1463-1476)
MJH_HD double ccdArea4(const double* a, const double* b, const double* c, const double* d) {
  double ad[3] = {d[0] - a[0], d[1] - a[1], d[2] - a[2]};
  double db[3] = {b[0] - d[0], b[1] - d[1], b[2] - d[2]};
  double bc[3] = {c[0] - b[0], c[1] - b[1], c[2] - b[2]};
  double ca[3] = {a[0] - c[0], a[1] - c[1], a[2] - c[2]};
  double e[3], f[3], g[3];
  cross(e, ad, db);
  cross(f, bc, ca);
  add3(g, e, f);
  return 0.5 * sqrt(dot3(g, g));
}

MJH_HD int ccdNext(int n, int i) { return i == n - 1 ? 0 : i + 1; }

// polygonQuad (:1491-1535), on vertex indices
MJH_HD void ccdPolygonQuad(int res[4], const double* P, int n) {
  int a = 0, b = 1, c = 2, d = 3;
  res[0] = a; res[1] = b; res[2] = c; res[3] = d;
  double m = ccdArea4(P + 3*a, P + 3*b, P + 3*c, P + 3*d), mn;
  for (; a < n; a++) {
    while (true) {
      mn = ccdArea4(P + 3*a, P + 3*b, P + 3*c, P + 3*ccdNext(n, d));
      if (mn <= m) break;
      m = mn;
      d = ccdNext(n, d);
      res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      while (true) {
        mn = ccdArea4(P + 3*a, P + 3*b, P + 3*ccdNext(n, c), P + 3*d);
        if (mn <= m) break;
        m = mn;
        c = ccdNext(n, c);
        res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      }
      while (true) {
        mn = ccdArea4(P + 3*a, P + 3*ccdNext(n, b), P + 3*c, P + 3*d);
        if (mn <= m) break;
        m = mn;
        b = ccdNext(n, b);
        res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      }
    }
    if (b == a) {
      b = ccdNext(n, b);
      if (c == b) {
        c = ccdNext(n, c);
        if (d == c) d = ccdNext(n, d);
      }
    }
  }
}

// the contact list of a multicontact call: x1 / x2 [3 CCD_MAXCON], nx
struct CcdContacts {
  double* x1;
  double* x2;
  int nx, maxc, bad;
  const mjhipModel* m;                                  // the mesh polygon data
};

// polygonClip (:1579-1690): face2 clipped by face1's edge planes (normal n), the vertices the
// contacts' x2, x1 = x2 - dir
MJH_HD void ccdPolygonClip(CcdContacts& C, const double* face1, int nf1, const double* face2,
                           int nf2, const double n[3], const double dir[3]) {
  if (nf1 < 3) return;
  if (nf1 > CCD_MAXFACE || nf2 > CCD_MAXFACE) {
    C.bad = 1;
    return;
  }
  double pn[3*CCD_MAXFACE], pd[CCD_MAXFACE];
  for (int i = 0; i < nf1; i++) {                       // planeNormal (:1540-1549)
    const double* v1 = face1 + 3*i;
    const double* v2 = face1 + 3*(i < nf1 - 1 ? i + 1 : 0);
    double v3[3], d1[3], d2[3];
    add3(v3, v1, n);
    sub3(d1, v2, v1);
    sub3(d2, v3, v1);
    cross(pn + 3*i, d1, d2);
    pd[i] = dot3(pn + 3*i, v1);
  }
  double buf[2][3*CCD_MAXPOLY];
  double* poly = buf[0];
  double* clip = buf[1];
  int np = nf2, nc = 0;
  for (int i = 0; i < nf2; i++) copy3(poly + 3*i, face2 + 3*i);
  for (int e = 0; e < nf1; e++) {
    const double* a = face1 + 3*e;
    for (int i = 0; i < np; i++) {
      const double* P = poly + 3*i;
      const double* Q = i < np - 1 ? poly + 3*(i + 1) : poly;
      const double dp[3] = {P[0] - a[0], P[1] - a[1], P[2] - a[2]};
      const double dq[3] = {Q[0] - a[0], Q[1] - a[1], Q[2] - a[2]};
      const bool in1 = dot3(dp, pn + 3*e) > 0, in2 = dot3(dq, pn + 3*e) > 0;   // halfspace
      if (!in1 && !in2) continue;
      if (nc + 2 > CCD_MAXPOLY) {                       // cannot happen for box faces
        C.bad = 1;
        return;
      }
      if (in1 && in2) {
        copy3(clip + 3*nc++, Q);
        continue;
      }
      // planeIntersect (:1561-1574)
      double ab[3];
      sub3(ab, Q, P);
      const double temp = dot3(pn + 3*e, ab);
      double t = mjhipMAXVAL;
      if (temp != 0.0) {
        t = (pd[e] - dot3(pn + 3*e, P)) / temp;
        if (t >= 0.0 && t <= 1.0) {
          double* r = clip + 3*nc;
          r[0] = P[0] + t*ab[0];
          r[1] = P[1] + t*ab[1];
          r[2] = P[2] + t*ab[2];
        }
      }
      nc++;
      if (t < 0.0 || t > 1.0) nc--;
      if (in2) copy3(clip + 3*nc++, Q);
    }
    double* tmp = poly;
    poly = clip;
    clip = tmp;
    np = nc;
    nc = 0;
  }
  if (np < 1) return;
  if (C.maxc < 5 && np > 4) {
    int rect[4];
    ccdPolygonQuad(rect, poly, np);
    C.nx = 4;
    for (int i = 0; i < 4; i++) {
      copy3(C.x2 + 3*i, poly + 3*rect[i]);
      sub3(C.x1 + 3*i, C.x2 + 3*i, dir);
    }
    return;
  }
  int k = 0;                                            // np <= CCD_MAXPOLY < mjMAXCONPAIR
  for (int i = 0; i < np; i++) {
    const double* q = poly + 3*i;
    bool skip = false;
    for (int j = 0; j < k && !skip; j++) {              // equal3 (:116-120)
      const double* x = C.x2 + 3*j;
      skip = fabs(x[0] - q[0]) < MINVAL && fabs(x[1] - q[1]) < MINVAL &&
             fabs(x[2] - q[2]) < MINVAL;
    }
    if (skip) continue;
    copy3(C.x2 + 3*k, q);
    sub3(C.x1 + 3*k, C.x2 + 3*k, dir);
    k++;
  }
  C.nx = k;
}

// globalcoord (:1695-1707)
MJH_HD void ccdGlobal(double r[3], const double mat[9], const double* pos, double l1,
                      double l2, double l3) {
  r[0] = mat[0]*l1 + mat[1]*l2 + mat[2]*l3;
  r[1] = mat[3]*l1 + mat[4]*l2 + mat[5]*l3;
  r[2] = mat[6]*l1 + mat[7]*l2 + mat[8]*l3;
  if (pos) {
    r[0] += pos[0];
    r[1] += pos[1];
    r[2] += pos[2];
  }
}

// the mesh vertex a support point is: the vertex whose global position (ccdToGlobal, as
// ccdMeshSupport forms it) equals p, or -1
MJH_HD int ccdMeshVertex(const CcdShape& s, const double* p) {
  for (int i = 0; i < s.nvert; i++) {
    const double t[3] = {(double)s.vert[3*i], (double)s.vert[3*i+1], (double)s.vert[3*i+2]};
    double r[3];
    ccdToGlobal(r, s.mat, t, s.pos);
    if (r[0] == p[0] && r[1] == p[1] && r[2] == p[2]) return i;
  }
  return -1;
}

// intersect (:1711-1723): up to 2 common entries of two arrays
MJH_HD int ccdIntersect(int res[2], const int* a, const int* b, int n, int k) {
  int count = 0;
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < k; j++) {
      if (a[i] == b[j]) {
        res[count++] = a[i];
        if (count == 2) return 2;
      }
    }
  }
  return count;
}

// meshNormals (:1727-1792): the normals of the mesh polygons through the feature's vertices;
// -1 when a vertex is on more than CCD_MAXFACE polygons
MJH_HD int ccdMeshNormals(const mjhipModel& m, double* res, int* ind, int dim,
                          const CcdShape& s, int v1, int v2, int v3) {
  const int polyadr = m.mesh_polyadr[s.meshid], vertadr = m.mesh_vertadr[s.meshid];
  const int* pm = m.mesh_polymap;
  if (dim == 3) {
    const int a1 = m.mesh_polymapadr[vertadr + v1], n1 = m.mesh_polymapnum[vertadr + v1];
    const int a2 = m.mesh_polymapadr[vertadr + v2], n2 = m.mesh_polymapnum[vertadr + v2];
    const int a3 = m.mesh_polymapadr[vertadr + v3], n3 = m.mesh_polymapnum[vertadr + v3];
    int edgeset[2], faceset[2];
    int n = ccdIntersect(edgeset, pm + a1, pm + a2, n1, n2);
    if (n == 0) return 0;
    n = ccdIntersect(faceset, edgeset, pm + a3, n, n3);
    if (n == 0) return 0;
    const double* nrm = m.mesh_polynormal + 3*(polyadr + faceset[0]);
    ccdGlobal(res, s.mat, nullptr, nrm[0], nrm[1], nrm[2]);
    ind[0] = faceset[0];
    return 1;
  }
  if (dim == 2) {
    const int a1 = m.mesh_polymapadr[vertadr + v1], n1 = m.mesh_polymapnum[vertadr + v1];
    const int a2 = m.mesh_polymapadr[vertadr + v2], n2 = m.mesh_polymapnum[vertadr + v2];
    int edgeset[2];
    const int n = ccdIntersect(edgeset, pm + a1, pm + a2, n1, n2);
    for (int i = 0; i < n; i++) {
      const double* nrm = m.mesh_polynormal + 3*(polyadr + edgeset[i]);
      ccdGlobal(res + 3*i, s.mat, nullptr, nrm[0], nrm[1], nrm[2]);
      ind[i] = edgeset[i];
    }
    return n;
  }
  if (dim == 1) {
    const int a1 = m.mesh_polymapadr[vertadr + v1];
    int n1 = m.mesh_polymapnum[vertadr + v1];
    if (n1 > 150) n1 = 150;                             // mjMAX_POLYVERT
    if (n1 > CCD_MAXFACE) return -1;
    for (int i = 0; i < n1; i++) {
      const int index = pm[a1 + i];
      const double* nrm = m.mesh_polynormal + 3*(polyadr + index);
      ccdGlobal(res + 3*i, s.mat, nullptr, nrm[0], nrm[1], nrm[2]);
      ind[i] = index;
    }
    return n1;
  }
  return 0;
}

// meshEdgeNormals (:1796-1842): the directions of the mesh edges from the feature's vertex;
// as in the reference, the edge's other end is read at the polygon-local position k of the
// previous vertex (verts + 3k), not at that vertex's id
MJH_HD int ccdMeshEdgeNormals(const mjhipModel& m, double* res, double* ends, int dim,
                              const CcdShape& s, const double* v1, const double* v2, int v1i) {
  if (dim == 2) {
    copy3(ends, v2);
    sub3(res, v2, v1);
    normalize3(res);
    return 1;
  }
  if (dim == 1) {
    const int polyadr = m.mesh_polyadr[s.meshid], vertadr = m.mesh_vertadr[s.meshid];
    const int a1 = m.mesh_polymapadr[vertadr + v1i];
    int n1 = m.mesh_polymapnum[vertadr + v1i];
    if (n1 > 150) n1 = 150;
    if (n1 > CCD_MAXFACE) return -1;
    for (int i = 0; i < n1; i++) {
      const int idx = m.mesh_polymap[a1 + i];
      const int adr = m.mesh_polyvertadr[polyadr + idx];
      const int nvert = m.mesh_polyvertnum[polyadr + idx];
      for (int j = 0; j < nvert; j++) {
        if (m.mesh_polyvert[adr + j] == v1i) {
          const float* vert = m.mesh_vert + 3*vertadr + 3*(j == 0 ? nvert - 1 : j - 1);
          ccdGlobal(ends + 3*i, s.mat, s.pos, vert[0], vert[1], vert[2]);
          sub3(res + 3*i, ends + 3*i, v1);
          normalize3(res + 3*i);
        }
      }
    }
    return n1;
  }
  return 0;
}

// meshFace (:1994-2015): polygon idx's vertices, in reverse order, in the global frame; -1
// for a polygon over CCD_MAXFACE vertices
MJH_HD int ccdMeshFace(const mjhipModel& m, double* res, const CcdShape& s, int idx) {
  const int polyadr = m.mesh_polyadr[s.meshid], vertadr = m.mesh_vertadr[s.meshid];
  const int adr = m.mesh_polyvertadr[polyadr + idx];
  int nvert = m.mesh_polyvertnum[polyadr + idx], j = 0;
  if (nvert > 150) nvert = 150;
  if (nvert > CCD_MAXFACE) return -1;
  for (int i = nvert - 1; i >= 0; i--) {
    const float* vert = m.mesh_vert + 3*vertadr + 3*m.mesh_polyvert[adr + i];
    ccdGlobal(res + 3*j++, s.mat, s.pos, vert[0], vert[1], vert[2]);
  }
  return nvert;
}

// boxNormals (:1846-1899)
MJH_HD int ccdBoxNormals(double res[9], int ind[3], int dim, const CcdShape& s, int v1, int v2,
                         int v3) {
  if (dim == 3) {
    const int x = ((v1 & 1) && (v2 & 1) && (v3 & 1)) - (!(v1 & 1) && !(v2 & 1) && !(v3 & 1));
    const int y = ((v1 & 2) && (v2 & 2) && (v3 & 2)) - (!(v1 & 2) && !(v2 & 2) && !(v3 & 2));
    const int z = ((v1 & 4) && (v2 & 4) && (v3 & 4)) - (!(v1 & 4) && !(v2 & 4) && !(v3 & 4));
    ccdGlobal(res, s.mat, nullptr, x, y, z);
    if (x) ind[0] = 0;
    if (y) ind[0] = 2;
    if (z) ind[0] = 4;
    if (x + y + z == -1) ind[0]++;
    return 1;
  }
  if (dim == 2) {
    const int x = ((v1 & 1) && (v2 & 1)) - (!(v1 & 1) && !(v2 & 1));
    const int y = ((v1 & 2) && (v2 & 2)) - (!(v1 & 2) && !(v2 & 2));
    const int z = ((v1 & 4) && (v2 & 4)) - (!(v1 & 4) && !(v2 & 4));
    if (x) {
      ccdGlobal(res, s.mat, nullptr, x, 0, 0);
      ind[0] = x > 0 ? 0 : 1;
    }
    if (y) {
      const int i = x ? 1 : 0;
      ccdGlobal(res + 3*i, s.mat, nullptr, 0, y, 0);
      ind[i] = y > 0 ? 2 : 3;
    }
    if (z) {
      ccdGlobal(res + 3, s.mat, nullptr, 0, 0, z);
      ind[1] = z > 0 ? 4 : 5;
    }
    return 2;
  }
  if (dim == 1) {
    const double x = (v1 & 1) ? 1 : -1, y = (v1 & 2) ? 1 : -1, z = (v1 & 4) ? 1 : -1;
    ccdGlobal(res, s.mat, nullptr, x, 0, 0);
    ccdGlobal(res + 3, s.mat, nullptr, 0, y, 0);
    ccdGlobal(res + 6, s.mat, nullptr, 0, 0, z);
    ind[0] = x > 0 ? 0 : 1;
    ind[1] = y > 0 ? 2 : 3;
    ind[2] = z > 0 ? 4 : 5;
    return 3;
  }
  return 0;
}

// boxEdgeNormals (:1903-1938)
MJH_HD int ccdBoxEdgeNormals(double res[9], double ends[9], int dim, const CcdShape& s,
                             const double* v1, const double* v2, int v1i) {
  if (dim == 2) {
    copy3(ends, v2);
    sub3(res, v2, v1);
    normalize3(res);
    return 1;
  }
  if (dim == 1) {
    const double x = (v1i & 1) ? s.size[0] : -s.size[0];
    const double y = (v1i & 2) ? s.size[1] : -s.size[1];
    const double z = (v1i & 4) ? s.size[2] : -s.size[2];
    ccdGlobal(ends, s.mat, s.pos, -x, y, z);
    sub3(res, ends, v1);
    normalize3(res);
    ccdGlobal(ends + 3, s.mat, s.pos, x, -y, z);
    sub3(res + 3, ends + 3, v1);
    normalize3(res + 3);
    ccdGlobal(ends + 6, s.mat, s.pos, x, y, -z);
    sub3(res + 6, ends + 6, v1);
    normalize3(res + 6);
    return 3;
  }
  return 0;
}

// boxFace (:1942-1990): the four corners of face idx (right, left, top, bottom, front, back)
MJH_HD int ccdBoxFace(double res[12], const CcdShape& s, int idx) {
  // corner sign bits per face vertex: x (1), y (2), z (4) positive
  constexpr unsigned char corner[6][4] = {{7, 3, 1, 5}, {2, 6, 4, 0}, {2, 3, 7, 6},
                                          {4, 5, 1, 0}, {6, 7, 5, 4}, {3, 2, 0, 1}};
  if (idx < 0 || idx > 5) return 0;
  for (int k = 0; k < 4; k++) {
    const int c = corner[idx][k];
    ccdGlobal(res + 3*k, s.mat, s.pos, (c & 1) ? s.size[0] : -s.size[0],
              (c & 2) ? s.size[1] : -s.size[1], (c & 4) ? s.size[2] : -s.size[2]);
  }
  return 4;
}

// simplexDim (:2052-2067)
MJH_HD int ccdSimplexDim(int* i1, int* i2, int* i3, const double** v1, const double** v2,
                         const double** v3) {
  const int a = *i1, b = *i2, c = *i3;
  if (a != b) return (c == a || c == b) ? 2 : 3;
  if (a != c) {
    *i2 = *i3;
    *v2 = *v3;
    return 2;
  }
  return 1;
}

// multicontact (:2071-2193) on the EPA's final face f, box and mesh pairs
template <int S>
MJH_HD void ccdMultiContact(const mjhipModel& m, CcdContacts& C, const CcdState& st,
                            const CcdMem<S>& M, int f, const CcdShape& A, const CcdShape& B) {
  const bool mesh1 = A.gtype == mjhipGEOM_MESH, mesh2 = B.gtype == mjhipGEOM_MESH;
  if ((!mesh1 && A.gtype != mjhipGEOM_BOX) || (!mesh2 && B.gtype != mjhipGEOM_BOX)) {
    C.bad = 1;                                          // not a box or mesh pair
    return;
  }
  SP<S, int> F = M.fint(f);
  double w[3][9];                                       // the face's vertices: v, p1, p2
  for (int k = 0; k < 3; k++) {
    SP<S> v = M.vtx(F[k]);
    for (int c = 0; c < 9; c++) w[k][c] = v[c];
  }
  auto corner = [&](const CcdShape& s, bool mesh, const double* p) MJH_LAMBDA_INLINE {
    return mesh ? ccdMeshVertex(s, p) : ccdBoxCorner(s, p);
  };
  int v11i = corner(A, mesh1, w[0] + 3), v12i = corner(A, mesh1, w[1] + 3);
  int v13i = corner(A, mesh1, w[2] + 3);
  int v21i = corner(B, mesh2, w[0] + 6), v22i = corner(B, mesh2, w[1] + 6);
  int v23i = corner(B, mesh2, w[2] + 6);
  if (v11i < 0 || v12i < 0 || v13i < 0 || v21i < 0 || v22i < 0 || v23i < 0) {
    C.bad = 1;                                          // a support point off the mesh's
    return;                                             // vertices (an inflated margin)
  }
  const double *v11 = w[0] + 3, *v12 = w[1] + 3, *v13 = w[2] + 3;
  const double *v21 = w[0] + 6, *v22 = w[1] + 6, *v23 = w[2] + 6;
  int nf1 = ccdSimplexDim(&v11i, &v12i, &v13i, &v11, &v12, &v13);
  int nf2 = ccdSimplexDim(&v21i, &v22i, &v23i, &v21, &v22, &v23);
  double n1[3*CCD_MAXFACE], n2[3*CCD_MAXFACE], ends[3*CCD_MAXFACE];
  double face1[3*CCD_MAXFACE], face2[3*CCD_MAXFACE];
  int idx1[CCD_MAXFACE], idx2[CCD_MAXFACE];
  int nn1 = mesh1 ? ccdMeshNormals(m, n1, idx1, nf1, A, v11i, v12i, v13i)
                  : ccdBoxNormals(n1, idx1, nf1, A, v11i, v12i, v13i);
  int nn2 = mesh2 ? ccdMeshNormals(m, n2, idx2, nf2, B, v21i, v22i, v23i)
                  : ccdBoxNormals(n2, idx2, nf2, B, v21i, v22i, v23i);
  if (nn1 < 0 || nn2 < 0) {
    C.bad = 1;
    return;
  }
  int i = 0, j = 0;
  bool found = false, edge1 = false, edge2 = false;
  for (int a = 0; a < nn1 && !found; a++) {             // alignedFaces (:2019-2031)
    for (int b = 0; b < nn2 && !found; b++) {
      if (dot3(n1 + 3*a, n2 + 3*b) < -CCD_FACE_TOL) {
        i = a;
        j = b;
        found = true;
      }
    }
  }
  // alignedFaceEdge (:2036-2048): the first (face, edge) pair within the tolerance
  auto faceEdge = [&](const double* edge, int ne, const double* face, int nfc) MJH_LAMBDA_INLINE {
    for (int a = 0; a < nfc; a++) {
      for (int b = 0; b < ne; b++) {
        if (fabs(dot3(edge + 3*b, face + 3*a)) < CCD_EDGE_TOL) {
          i = b;
          j = a;
          return true;
        }
      }
    }
    return false;
  };
  if (!found) {
    if (nf1 < 3 && nf1 <= nf2) {
      nn1 = mesh1 ? ccdMeshEdgeNormals(m, n1, ends, nf1, A, v11, v12, v11i)
                  : ccdBoxEdgeNormals(n1, ends, nf1, A, v11, v12, v11i);
      if (nn1 < 0) {
        C.bad = 1;
        return;
      }
      if (!faceEdge(n1, nn1, n2, nn2)) return;
      edge1 = true;
    } else if (nf2 < 3) {
      nn2 = mesh2 ? ccdMeshEdgeNormals(m, n2, ends, nf2, B, v21, v22, v21i)
                  : ccdBoxEdgeNormals(n2, ends, nf2, B, v21, v22, v21i);
      if (nn2 < 0) {
        C.bad = 1;
        return;
      }
      if (!faceEdge(n2, nn2, n1, nn1)) return;
      edge2 = true;
    } else {
      return;
    }
  }
  if (edge1) {
    copy3(face1, w[0] + 3);
    copy3(face1 + 3, ends + 3*i);
    nf1 = 2;
  } else {
    const int ind = edge2 ? idx1[j] : idx1[i];
    nf1 = mesh1 ? ccdMeshFace(m, face1, A, ind) : ccdBoxFace(face1, A, ind);
  }
  if (edge2) {
    copy3(face2, w[0] + 6);
    copy3(face2 + 3, ends + 3*i);
    nf2 = 2;
  } else {
    nf2 = mesh2 ? ccdMeshFace(m, face2, B, idx2[j]) : ccdBoxFace(face2, B, idx2[j]);
  }
  if (nf1 < 0 || nf2 < 0) {
    C.bad = 1;
    return;
  }
  double diff[3], dir[3];
  sub3(diff, st.x2, st.x1);
  const double nd = sqrt(dot3(diff, diff));
  if (edge1) {
    scl3(dir, n2 + 3*j, nd);
    ccdPolygonClip(C, face2, nf2, face1, nf1, n2 + 3*j, dir);
  } else if (edge2) {
    scl3(dir, n1 + 3*j, -nd);
    ccdPolygonClip(C, face1, nf1, face2, nf2, n1 + 3*j, dir);
  } else {
    scl3(dir, n2 + 3*j, nd);
    ccdPolygonClip(C, face1, nf1, face2, nf2, n1 + 3*i, dir);
  }
}

// mjc_ccd (:2215-2343) with max_contacts `maxc` (1: mjc_Convex and mj_geomDistanceCCD; 0: the
// distance alone, no penetration recovery, mjhip_ccdBatch) and the distance cutoff `cutoff`
// (0 for mjc_Convex's contacts, the bound for mj_geomDistanceCCD)
template <int S, bool MULTI = false>
MJH_HD double ccdRun(CcdState& st, const CcdMem<S>& M, CcdShape& A, CcdShape& B, int kmax,
                     double tol, double cutoff, int maxc = 1, CcdContacts* multi = nullptr) {
  ccdCenter(st.x1, A);
  ccdCenter(st.x2, B);
  st.iters = 0;
  st.tol = tol;
  st.kmax = kmax;
  st.cutoff = cutoff;
  st.unsupported = 0;
  const bool shrinkA = A.gtype == mjhipGEOM_SPHERE || A.gtype == mjhipGEOM_CAPSULE;
  const bool shrinkB = B.gtype == mjhipGEOM_SPHERE || B.gtype == mjhipGEOM_CAPSULE;
  if (shrinkA || shrinkB) {
    double full1 = 0, full2 = 0;
    const double m1 = A.margin, m2 = B.margin;
    if (shrinkA) {
      full1 = A.size[0] + 0.5*m1;
      A.kind = A.gtype == mjhipGEOM_SPHERE ? CCD_POINT : CCD_LINE;
      A.margin = 0;
    }
    if (shrinkB) {
      full2 = B.size[0] + 0.5*m2;
      B.kind = B.gtype == mjhipGEOM_SPHERE ? CCD_POINT : CCD_LINE;
      B.margin = 0;
    }
    st.cutoff += full1 + full2;
    ccdGjk(st, M, A, B);
    st.cutoff = cutoff;
    A.margin = m1;
    B.margin = m2;
    A.kind = A.gtype;
    B.kind = B.gtype;
    if (st.dist > st.tol) {                             // shallow: inflate (:2195-2210)
      double n[3];
      sub3(n, st.x2, st.x1);
      normalize3(n);
      if (full1) {
        st.x1[0] += full1*n[0]; st.x1[1] += full1*n[1]; st.x1[2] += full1*n[2];
      }
      if (full2) {
        st.x2[0] -= full2*n[0]; st.x2[1] -= full2*n[1]; st.x2[2] -= full2*n[2];
      }
      st.dist -= (full1 + full2);
      if (st.dist > st.cutoff) st.dist = mjhipMAXVAL;
      return st.dist;
    }
    if (!maxc) {                                        // contact not needed
      st.nx = 0;
      st.dist = 0;
      return 0;
    }
    st.iters = 0;
    ccdCenter(st.x1, A);
    ccdCenter(st.x2, B);
  }
  ccdGjk(st, M, A, B);
  if (!maxc) return st.dist;                            // no penetration recovery
  if (st.dist <= tol && st.nsimplex > 1) {
    st.dist = 0;
    CcdPoly P{0, 0, 0, 0};
    const int ret = st.nsimplex == 2 ? ccdFromSegment(M, P, st, A, B) :
                    st.nsimplex == 3 ? ccdFromTriangle(M, P, st, A, B) :
                                       ccdFromTetra(M, P, st, A, B);
    if (!ret) {
      const int f = ccdEpa(st, M, P, A, B);
      if (MULTI && maxc > 1 && f >= 0) ccdMultiContact(*multi->m, *multi, st, M, f, A, B);
    }
  }
  return st.dist;
}

// the mesh fields of a geom's solver object (mjc_initCCDObj :716-743)
MJH_HD void ccdMeshData(CcdShape& s, const mjhipModel& m, int g) {
  s.vert = nullptr;
  s.graph = nullptr;
  s.nvert = 0;
  s.vertindex = s.meshindex = -1;
  s.meshid = -1;
  if (s.gtype == mjhipGEOM_MESH) {
    const int id = m.geom_dataid[g];
    s.meshid = id;
    s.vert = m.mesh_vert + 3*m.mesh_vertadr[id];
    s.nvert = m.mesh_vertnum[id];
    s.graph = m.mesh_graphadr[id] >= 0 ? m.mesh_graph + m.mesh_graphadr[id] : nullptr;
  }
}

template <int S>
MJH_HD void ccdShape(CcdShape& s, const mjhipModel& m, const Lane<S>& d, int g, double margin) {
  s.kind = s.gtype = m.geom_type[g];
  for (int k = 0; k < 3; k++) s.pos[k] = d.geom_xpos[3*g + k];
  for (int k = 0; k < 9; k++) s.mat[k] = d.geom_xmat[9*g + k];
  for (int k = 0; k < 3; k++) s.size[k] = m.geom_size[3*g + k];
  s.margin = margin;
  ccdMeshData(s, m, g);
}

// scratch of one standalone mjc_ccd call with max_iterations N (ccdGeneral): the CcdMem
// layout of the mirror's ccd / ccdi fields with the face capacity 6 N + 6
MJH_HD long ccdScratchDoubles(int N) { return 72 + 9L*(5 + N) + 5L*(6*N + 6); }
MJH_HD long ccdScratchInts(int N) { return 13L*(6*N + 6); }

// mjc_ccd (engine_collision_gjk.c:2215-2343, MJAPI) as the reference's own tests call it
// (engine_collision_gjk_test.cc:62-84 GeomDist, :86-150 Penetration): geoms g1, g2 of m at the
// given frames, object margin `margin` on both (mjc_initCCDObj), config {N, tol, maxc,
// cutoff}, contiguous scratch x / xi (ccdScratchDoubles / Ints). out (2 + 6 CCD_MAXCON): dist,
// nx, x1[3 CCD_MAXCON], x2[3 CCD_MAXCON]; MULTI: maxc > 1 runs multicontact. Returns 0, 1
// when the polytope outgrew the face capacity, 2 for a multicontact outside the built subset
// (a mesh).
template <bool MULTI = false>
MJH_HD int ccdGeneral(const mjhipModel& m, int g1, int g2, const double* pos1,
                      const double* mat1, const double* pos2, const double* mat2,
                      double margin, int N, double tol, int maxc, double cutoff, double* x,
                      int* xi, double* out) {
  CcdMem<1> M{{x}, {xi}, 5 + N, 6*N + 6};
  CcdShape sh[2];
  const int g[2] = {g1, g2};
  const double* pos[2] = {pos1, pos2};
  const double* mat[2] = {mat1, mat2};
  for (int j = 0; j < 2; j++) {
    CcdShape& s = sh[j];
    s.kind = s.gtype = m.geom_type[g[j]];
    for (int k = 0; k < 3; k++) s.pos[k] = pos[j][k];
    for (int k = 0; k < 9; k++) s.mat[k] = mat[j][k];
    for (int k = 0; k < 3; k++) s.size[k] = m.geom_size[3*g[j] + k];
    s.margin = margin;
    ccdMeshData(s, m, g[j]);
  }
  CcdState st;
  st.nx = 0;
  CcdContacts C{out + 2, out + 2 + 3*CCD_MAXCON, 0, maxc, 0, &m};
  const double dist = ccdRun<1, MULTI>(st, M, sh[0], sh[1], N, tol, cutoff, maxc, &C);
  out[0] = dist;
  if (MULTI && C.nx) {
    out[1] = C.nx;                                      // the polygon's contacts, in place
  } else {
    out[1] = st.nx;
    for (int k = 0; k < 3; k++) {
      out[2 + k] = st.x1[k];
      out[2 + 3*CCD_MAXCON + k] = st.x2[k];
    }
  }
  return st.unsupported ? 1 : (C.bad ? 2 : 0);
}

// mjc_CCDIteration (convex.c:792-819) on the shapes' current frames: 0 or 1 contacts
template <int S>
MJH_HD int ccdIteration(RawContact& c, const mjhipModel& m, const CcdMem<S>& M, CcdShape& A,
                        CcdShape& B, double margin, int* status) {
  CcdState st;
  const double dist = ccdRun(st, M, A, B, m.opt.ccd_iterations, m.opt.ccd_tolerance, 0.0);
  if (st.unsupported) {
    *status |= MJHIP_INST_UNSUPPORTED;
    return 0;
  }
  if (!(dist < 0) || st.nx < 1) return 0;
  c.dist = margin + dist;
  c.frame[0] = st.x1[0] - st.x2[0];
  c.frame[1] = st.x1[1] - st.x2[1];
  c.frame[2] = st.x1[2] - st.x2[2];
  normalize3(c.frame);
  c.pos[0] = 0.5*(st.x1[0] + st.x2[0]);
  c.pos[1] = 0.5*(st.x1[1] + st.x2[1]);
  c.pos[2] = 0.5*(st.x1[2] + st.x2[2]);
  for (int k = 3; k < 9; k++) c.frame[k] = 0;
  return 1;
}

// mjc_Convex through mjc_CCDIteration (convex.c:792-819, :915-1001): 0 or 1 contacts
template <int S>
MJH_HD int colConvex(RawContact& c, const mjhipModel& m, const Lane<S>& d, int g1, int g2,
                     double margin, int* status) {
  CcdMem<1> M{{d.ccdx}, {d.ccdxi}, 5 + m.opt.ccd_iterations, mjh_ccdFaceCap(&m)};
  CcdShape A, B;
  ccdShape(A, m, d, g1, margin);
  ccdShape(B, m, d, g2, margin);
  return ccdIteration(c, m, M, A, B, margin, status);
}

// mju_rotateFrame (convex.c:862-880): the frame rotated by rot about origin
MJH_HD void ccdRotateFrame(const double origin[3], const double rot[9], double xmat[9],
                           double xpos[3]) {
  double mat[9], vec[3], rel[3];
  for (int i = 0; i < 3; i++) {           // mju_mulMatMat3 (engine_util_blas.c:193-203)
    for (int j = 0; j < 3; j++) {
      mat[3*i+j] = rot[3*i]*xmat[j] + rot[3*i+1]*xmat[3+j] + rot[3*i+2]*xmat[6+j];
    }
  }
  for (int k = 0; k < 9; k++) xmat[k] = mat[k];
  sub3(rel, origin, xpos);
  mulMatVec3(vec, rot, rel);
  sub3(vec, vec, rel);
  sub3(xpos, xpos, vec);
}

// mjc_Convex with mjENBL_MULTICCD (convex.c:915-1001) for a pair without a sphere or an
// ellipsoid. A box / mesh pair without margin (singlePass :895-909) asks mjc_ccd for up to 4
// contacts -- the multicontact polygon (ccdMultiContact), or the one EPA contact -- and stops
// there. Other pairs: the first contact, then the four perturbed ones (:933-999) -- both geoms rotated
// about the first contact by -+1e-3 rad around its frame's y and z axes (geom 2 by the
// inverse), each new contact farther than 1e-3 min(rbound) from all earlier ones kept with
// the first one's depth -- handed to `store` in order (false: the list is full). The frames
// are perturbed on the solver's own copies (the reference rotates mjData's and restores
// them). sin / cos of the half angle are the correctly rounded constants, so the device
// libm cannot move a last bit.
template <int S, class Store>
MJH_HD void colConvexMulti(const mjhipModel& m, const Lane<S>& d, int g1, int g2,
                           double margin, int* status, Store store) {
  CcdMem<1> M{{d.ccdx}, {d.ccdxi}, 5 + m.opt.ccd_iterations, mjh_ccdFaceCap(&m)};
  CcdShape A, B;
  ccdShape(A, m, d, g1, margin);
  ccdShape(B, m, d, g2, margin);
  if (margin <= 0 && (A.gtype == mjhipGEOM_BOX || A.gtype == mjhipGEOM_MESH) &&
      (B.gtype == mjhipGEOM_BOX || B.gtype == mjhipGEOM_MESH)) {
    double x1[12], x2[12];                              // max_contacts 4: at most 4 contacts
    CcdContacts C{x1, x2, 0, 4, 0, &m};
    CcdState st;
    const double dist = ccdRun<1, true>(st, M, A, B, m.opt.ccd_iterations,
                                        m.opt.ccd_tolerance, 0.0, 4, &C);
    if (st.unsupported || C.bad) {
      *status |= MJHIP_INST_UNSUPPORTED;
      return;
    }
    if (!(dist < 0)) return;
    const int n = C.nx ? C.nx : st.nx;
    for (int i = 0; i < n; i++) {
      const double* a = C.nx ? x1 + 3*i : st.x1;
      const double* b = C.nx ? x2 + 3*i : st.x2;
      RawContact c;
      c.dist = margin + dist;
      c.frame[0] = a[0] - b[0];
      c.frame[1] = a[1] - b[1];
      c.frame[2] = a[2] - b[2];
      normalize3(c.frame);
      c.pos[0] = 0.5*(a[0] + b[0]);
      c.pos[1] = 0.5*(a[1] + b[1]);
      c.pos[2] = 0.5*(a[2] + b[2]);
      for (int k = 3; k < 9; k++) c.frame[k] = 0;
      if (!store(c)) return;
    }
    return;
  }
  RawContact c0;
  if (!ccdIteration(c0, m, M, A, B, margin, status)) return;
  if (!store(c0)) return;
  double frame[9];
  for (int k = 0; k < 9; k++) frame[k] = c0.frame[k];
  makeFrame(frame);
  const double rb1 = m.geom_rbound[g1], rb2 = m.geom_rbound[g2];
  const double tolerance = 1e-3 * (rb1 < rb2 ? rb1 : rb2);
  double p1[3], r1[9], p2[3], r2[9];
  copy3(p1, A.pos);
  copy3(p2, B.pos);
  for (int k = 0; k < 9; k++) { r1[k] = A.mat[k]; r2[k] = B.mat[k]; }
  double kept[5][3];
  copy3(kept[0], c0.pos);
  int ncon = 1;
  constexpr double kSin = 0.0004999999791666669;   // sin(1e-3 / 2)
  constexpr double kCos = 0.9999998750000026;      // cos(1e-3 / 2)
  for (int ai = 0; ai < 2; ai++) {
    const double* axis = frame + 3 + 3*ai;
    for (int gi = 0; gi < 2; gi++) {
      const double s = gi ? kSin : -kSin;               // angles {-1e-3, 1e-3}
      const double quat[4] = {kCos, axis[0]*s, axis[1]*s, axis[2]*s};   // axisAngle2Quat
      double rot[9], inv[9];
      quat2Mat(rot, quat);
      ccdRotateFrame(c0.pos, rot, A.mat, A.pos);
      for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) inv[3*j+i] = rot[3*i+j];
      }
      ccdRotateFrame(c0.pos, inv, B.mat, B.pos);
      RawContact ck;
      bool fresh = ccdIteration(ck, m, M, A, B, margin, status) != 0;
      for (int i = 0; i < ncon && fresh; i++) {          // mjc_isDistinctContact (:851-858)
        double dif[3];
        sub3(dif, kept[i], ck.pos);
        if (sqrt(dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2]) <= tolerance) fresh = false;
      }
      if (fresh) {
        ck.dist = c0.dist;
        copy3(kept[ncon], ck.pos);
        ncon++;
        if (!store(ck)) return;
      }
      copy3(A.pos, p1);
      copy3(B.pos, p2);
      for (int k = 0; k < 9; k++) { A.mat[k] = r1[k]; B.mat[k] = r2[k]; }
    }
  }
}

// the pair runs MULTICCD (colConvexMulti): a convex pair without a sphere or an ellipsoid
// with the flag on
MJH_HD bool multiCcdPair(const mjhipModel& m, int t1, int t2) {
  return (m.opt.enableflags & mjhipENBL_MULTICCD) && mjhip_isConvexPair(t1, t2) &&
         t1 != mjhipGEOM_SPHERE && t1 != mjhipGEOM_ELLIPSOID && t2 != mjhipGEOM_ELLIPSOID;
}

// mjc_PlaneConvex (convex.c:1045-1080) for an ellipsoid: the libccd support (mjccd_support
// :501-704) at -normal, object margin 0, one contact
template <class P1, class M1, class P2, class M2>
MJH_HD int colPlaneEllipsoid(RawContact& c, double margin, P1 pos1, M1 mat1, P2 pos2, M2 mat2,
                             const double size[3]) {
  const double normal[3] = {mat1[2], mat1[5], mat1[8]};
  const double dir[3] = {-mat1[2], -mat1[5], -mat1[8]};
  double ld[3], v[3], dif[3];
  mulMatTVec3(ld, mat2, dir);
  for (int i = 0; i < 3; i++) v[i] = ld[i]*size[i];
  normalize3(v);
  for (int i = 0; i < 3; i++) v[i] *= size[i];
  for (int i = 0; i < 3; i++) v[i] += ld[i]*0.0/2;
  mulMatVec3(v, mat2, v);
  addTo3(v, pos2);
  sub3(dif, v, pos1);
  const double dist = dot3(normal, dif);
  if (dist > margin) return 0;
  c.dist = dist;
  copy3(c.pos, v);
  addToScl3(c.pos, normal, -0.5*dist);
  copy3(c.frame, normal);
  for (int k = 3; k < 9; k++) c.frame[k] = 0;
  return 1;
}

// mjccd_support (convex.c:501-704), the libccd-style support of a geom at unit direction dir
// in its current frame (s.pos / s.mat): a mesh hill-climbs from s.meshindex with the start
// vertex's own value as the first bound and records the result in s.meshindex; the result is
// inflated by half the object's margin
MJH_HD void ccdSupportLib(double r[3], CcdShape& s, const double dir[3]) {
  double ld[3], res[3];
  mulMatTVec3(ld, s.mat, dir);
  const double* size = s.size;
  const int t = s.gtype;
  if (t == mjhipGEOM_SPHERE) {
    scl3(res, ld, size[0]);
  } else if (t == mjhipGEOM_CAPSULE) {
    scl3(res, ld, size[0]);
    res[2] += (ld[2] < 0 ? -1.0 : (ld[2] > 0 ? 1.0 : 0.0)) * size[1];
  } else if (t == mjhipGEOM_ELLIPSOID) {
    for (int i = 0; i < 3; i++) res[i] = ld[i] * size[i];
    normalize3(res);
    for (int i = 0; i < 3; i++) res[i] *= size[i];
  } else if (t == mjhipGEOM_CYLINDER) {
    const double tmp = sqrt(ld[0]*ld[0] + ld[1]*ld[1]);
    if (tmp > MINVAL) {
      res[0] = ld[0]/tmp*size[0];
      res[1] = ld[1]/tmp*size[0];
    } else {
      res[0] = res[1] = 0;
    }
    res[2] = (ld[2] < 0 ? -1.0 : (ld[2] > 0 ? 1.0 : 0.0)) * size[1];
  } else if (t == mjhipGEOM_BOX) {
    for (int i = 0; i < 3; i++) res[i] = (ld[i] < 0 ? -1.0 : (ld[i] > 0 ? 1.0 : 0.0)) * size[i];
  } else {                                  // mesh
    const float* V = s.vert;
    double tmp = -1E+10;
    int ibest = -1;
    if (!s.graph) {
      for (int i = 0; i < s.nvert; i++) {
        const double vdot = ld[0]*(double)V[3*i] + ld[1]*(double)V[3*i+1] +
                            ld[2]*(double)V[3*i+2];
        if (vdot > tmp) {
          tmp = vdot;
          ibest = i;
        }
      }
      s.meshindex = ibest;
    } else {
      const int numvert = s.graph[0];
      const int* edgeadr = s.graph + 2;
      const int* globalid = s.graph + 2 + numvert;
      const int* localid = s.graph + 2 + 2*numvert;
      ibest = s.meshindex < 0 ? 0 : s.meshindex;
      const float* vb = V + 3*globalid[ibest];
      tmp = ld[0]*(double)vb[0] + ld[1]*(double)vb[1] + ld[2]*(double)vb[2];
      int change = 1, locid;
      while (change) {
        change = 0;
        int i = edgeadr[ibest];
        while ((locid = localid[i]) >= 0) {
          const float* vx = V + 3*globalid[locid];
          const double vdot = ld[0]*(double)vx[0] + ld[1]*(double)vx[1] + ld[2]*(double)vx[2];
          if (vdot > tmp) {
            tmp = vdot;
            ibest = locid;
            change = 1;
          }
          i++;
        }
      }
      s.meshindex = ibest;
      ibest = globalid[ibest];
    }
    if (ibest < 0) {
      res[0] = res[1] = res[2] = 0;
    } else {
      for (int i = 0; i < 3; i++) res[i] = (double)V[3*ibest + i];
    }
  }
  for (int i = 0; i < 3; i++) res[i] += ld[i] * s.margin/2;
  mulMatVec3(res, s.mat, res);
  addTo3(res, s.pos);
  copy3(r, res);
}

// addplanemesh (convex.c:1010-1040)
MJH_HD bool planeMeshContact(RawContact& c, const float* vertex, const double pos1[3],
                             const double normal1[3], const double pos2[3],
                             const double mat2[9], const double first[3], double rbound) {
  double pnt[3], v[3] = {vertex[0], vertex[1], vertex[2]}, dif[3];
  mulMatVec3(pnt, mat2, v);
  addTo3(pnt, pos2);
  const double dd[3] = {pnt[0] - first[0], pnt[1] - first[1], pnt[2] - first[2]};
  if (sqrt(dd[0]*dd[0] + dd[1]*dd[1] + dd[2]*dd[2]) < 0.3*rbound) return false;
  sub3(dif, pnt, pos1);
  c.dist = dot3(normal1, dif);
  copy3(c.pos, pnt);
  addToScl3(c.pos, normal1, -0.5*c.dist);
  copy3(c.frame, normal1);
  for (int k = 3; k < 9; k++) c.frame[k] = 0;
  return true;
}

// mjc_PlaneConvex (convex.c:1045-1141) for a mesh: the libccd support at -normal gives the
// first contact, then up to maxplanemesh = 3 in all with the vertices below the margin around
// the support vertex (its hull-graph neighbours, else every vertex); each contact goes to
// emit as it is made
template <int S, class Emit>
MJH_HD void colPlaneMesh(const mjhipModel& m, const Lane<S>& d, int g1, int g2, double margin,
                         Emit&& emit) {
  double pos1[3], mat1[9], pos2[3], mat2[9];
  for (int k = 0; k < 3; k++) { pos1[k] = d.gxpos[3*g1 + k]; pos2[k] = d.gxpos[3*g2 + k]; }
  for (int k = 0; k < 9; k++) { mat1[k] = d.geom_xmat[9*g1 + k]; mat2[k] = d.geom_xmat[9*g2 + k]; }
  const double normal[3] = {mat1[2], mat1[5], mat1[8]};
  const double dir[3] = {-mat1[2], -mat1[5], -mat1[8]};
  CcdShape obj;
  obj.kind = obj.gtype = mjhipGEOM_MESH;
  copy3(obj.pos, pos2);
  for (int k = 0; k < 9; k++) obj.mat[k] = mat2[k];
  for (int k = 0; k < 3; k++) obj.size[k] = m.geom_size[3*g2 + k];
  obj.margin = 0;
  ccdMeshData(obj, m, g2);
  double v[3], dif[3];
  ccdSupportLib(v, obj, dir);
  sub3(dif, v, pos1);
  const double dist = dot3(normal, dif);
  if (dist > margin) return;
  RawContact c;
  c.dist = dist;
  copy3(c.pos, v);
  addToScl3(c.pos, normal, -0.5*dist);
  copy3(c.frame, normal);
  for (int k = 3; k < 9; k++) c.frame[k] = 0;
  const double first[3] = {c.pos[0], c.pos[1], c.pos[2]};
  if (!emit(c)) return;
  int count = 1;
  const int id = m.geom_dataid[g2];
  const float* vertdata = m.mesh_vert + 3*m.mesh_vertadr[id];
  double locdir[3];
  mulMatTVec3(locdir, mat2, dir);
  sub3(dif, pos2, pos1);
  const double threshold = dot3(normal, dif) - margin;
  const double rbound = m.geom_rbound[g2];
  if (m.mesh_graphadr[id] < 0) {
    for (int i = 0; i < m.mesh_vertnum[id] && count < 3; i++) {
      const float* vx = vertdata + 3*i;
      const double vdot = locdir[0]*(double)vx[0] + locdir[1]*(double)vx[1] +
                          locdir[2]*(double)vx[2];
      if (vdot > threshold && i != obj.meshindex) {
        RawContact e;
        if (planeMeshContact(e, vx, pos1, normal, pos2, mat2, first, rbound)) {
          count++;
          if (!emit(e)) return;
        }
      }
    }
  } else if (obj.meshindex >= 0) {
    const int* graph = m.mesh_graph + m.mesh_graphadr[id];
    const int numvert = graph[0];
    const int* edgeadr = graph + 2;
    const int* globalid = graph + 2 + numvert;
    const int* localid = graph + 2 + 2*numvert;
    int i = edgeadr[obj.meshindex], locid;
    while ((locid = localid[i]) >= 0 && count < 3) {
      const float* vx = vertdata + 3*globalid[locid];
      const double vdot = locdir[0]*(double)vx[0] + locdir[1]*(double)vx[1] +
                          locdir[2]*(double)vx[2];
      if (vdot > threshold) {
        RawContact e;
        if (planeMeshContact(e, vx, pos1, normal, pos2, mat2, first, rbound)) {
          count++;
          if (!emit(e)) return;
        }
      }
      i++;
    }
  }
}

// mjc_ellipsoidInside (convex.c:1363-1414) and mjc_ellipsoidOutside (:1419-1464)
MJH_HD int ellipsoidInside(double nrm[3], const double pos[3], const double size[3]) {
  const double S2inv[3] = {1/(size[0]*size[0]), 1/(size[1]*size[1]), 1/(size[2]*size[2])};
  const double C = pos[0]*pos[0]*S2inv[0] + pos[1]*pos[1]*S2inv[1] + pos[2]*pos[2]*S2inv[2] - 1;
  if (C > 0) return 0;
  normalize3(nrm);
  for (int iter = 0; iter < 30; iter++) {
    const double A = nrm[0]*nrm[0]*S2inv[0] + nrm[1]*nrm[1]*S2inv[1] + nrm[2]*nrm[2]*S2inv[2];
    const double B = pos[0]*nrm[0]*S2inv[0] + pos[1]*nrm[1]*S2inv[1] + pos[2]*nrm[2]*S2inv[2];
    const double det = B*B - A*C;
    if (det < MINVAL || A < MINVAL) return iter > 0;
    const double x = (-B + sqrt(det))/A;
    if (x < 0) return iter > 0;
    double pnt[3];
    for (int k = 0; k < 3; k++) pnt[k] = pos[k] + nrm[k]*x;   // mju_addScl3
    double nn[3] = {pnt[0]*S2inv[0], pnt[1]*S2inv[1], pnt[2]*S2inv[2]};
    normalize3(nn);
    const double dd[3] = {nrm[0] - nn[0], nrm[1] - nn[1], nrm[2] - nn[2]};
    const double change = sqrt(dd[0]*dd[0] + dd[1]*dd[1] + dd[2]*dd[2]);
    copy3(nrm, nn);
    if (change < 1e-6) break;
  }
  return 1;
}

MJH_HD int ellipsoidOutside(double nrm[3], const double pos[3], const double size[3]) {
  const double S2[3] = {size[0]*size[0], size[1]*size[1], size[2]*size[2]};
  const double PS2[3] = {pos[0]*pos[0]*S2[0], pos[1]*pos[1]*S2[1], pos[2]*pos[2]*S2[2]};
  double la = 0;
  for (int iter = 0; iter < 30; iter++) {
    const double R[3] = {1/(S2[0]+la), 1/(S2[1]+la), 1/(S2[2]+la)};
    const double val = PS2[0]*R[0]*R[0] + PS2[1]*R[1]*R[1] + PS2[2]*R[2]*R[2] - 1;
    if (val < 1e-6) break;
    const double deriv = -2*(PS2[0]*R[0]*R[0]*R[0] + PS2[1]*R[1]*R[1]*R[1] +
                             PS2[2]*R[2]*R[2]*R[2]);
    if (deriv > -MINVAL) break;
    const double delta = -val/deriv;
    if (delta < 1e-6) break;
    la += delta;
  }
  nrm[0] = pos[0]/(S2[0]+la);
  nrm[1] = pos[1]/(S2[1]+la);
  nrm[2] = pos[2]/(S2[2]+la);
  normalize3(nrm);
  return 1;
}

// mjc_fixNormal (convex.c:1469-1614): the contact normal from the smooth geom's surface
template <int S>
MJH_HD void fixNormal(const mjhipModel& m, const Lane<S>& d, RawContact& con, int g1, int g2) {
  const int gid[2] = {g1, g2};
  int type[2];
  for (int i = 0; i < 2; i++) {
    type[i] = m.geom_type[gid[i]];
    if (type[i] != mjhipGEOM_SPHERE && type[i] != mjhipGEOM_CAPSULE &&
        type[i] != mjhipGEOM_ELLIPSOID && type[i] != mjhipGEOM_CYLINDER) {
      type[i] = -1;
    }
  }
  if (type[0] == -1 && type[1] == -1) return;
  double normal[2][3] = {{con.frame[0], con.frame[1], con.frame[2]},
                         {-con.frame[0], -con.frame[1], -con.frame[2]}};
  int processed[2] = {0, 0};
  for (int i = 0; i < 2; i++) {
    if (type[i] == -1) continue;
    double mat[9], gp[3];
    for (int k = 0; k < 9; k++) mat[k] = d.geom_xmat[9*gid[i] + k];
    for (int k = 0; k < 3; k++) gp[k] = d.gxpos[3*gid[i] + k];
    const double* size = m.geom_size + 3*gid[i];
    double dif[3], pos[3], nrm[3], dst1, dst2;
    sub3(dif, con.pos, gp);
    mulMatTVec3(pos, mat, dif);
    mulMatTVec3(nrm, mat, normal[i]);
    if (type[i] == mjhipGEOM_SPHERE) {
      copy3(nrm, pos);
      processed[i] = 1;
    } else if (type[i] == mjhipGEOM_CAPSULE) {
      if (pos[2] < -size[1]) {
        nrm[2] = pos[2] + size[1];
      } else if (pos[2] > size[1]) {
        nrm[2] = pos[2] - size[1];
      } else {
        nrm[2] = 0;
      }
      nrm[0] = pos[0];
      nrm[1] = pos[1];
      processed[i] = 1;
    } else if (type[i] == mjhipGEOM_ELLIPSOID) {
      if (!(size[0] < MINVAL || size[1] < MINVAL || size[2] < MINVAL)) {
        dst1 = pos[0]*pos[0]/(size[0]*size[0]) + pos[1]*pos[1]/(size[1]*size[1]) +
               pos[2]*pos[2]/(size[2]*size[2]);
        processed[i] = dst1 <= 1 ? ellipsoidInside(nrm, pos, size)
                                 : ellipsoidOutside(nrm, pos, size);
      }
    } else {                                // cylinder
      if (!(fabs(pos[2]) > 0.95*size[1])) {
        dst1 = fabs(size[1] - fabs(pos[2]));
        dst2 = fabs(size[0] - sqrt(pos[0]*pos[0] + pos[1]*pos[1]));
        if (!(dst1 < 0.25*dst2)) {
          nrm[0] = pos[0];
          nrm[1] = pos[1];
          nrm[2] = 0;
          processed[i] = 1;
        }
      }
    }
    if (processed[i]) {
      normalize3(nrm);
      mulMatVec3(normal[i], mat, nrm);
    }
  }
  if (processed[0] && processed[1]) {
    sub3(con.frame, normal[0], normal[1]);
    normalize3(con.frame);
  } else if (processed[0]) {
    copy3(con.frame, normal[0]);
  } else if (processed[1]) {
    scl3(con.frame, normal[1], -1);
  }
  if (processed[0] || processed[1]) {
    for (int k = 3; k < 6; k++) con.frame[k] = 0;
  }
}

// addVert (convex.c:1154-1168) on the compressed prism
MJH_HD void prismAddVert(int& nvert, CcdShape& s, double x, double y, double z) {
  s.px[0] = s.px[1]; s.py[0] = s.py[1]; s.pzt[0] = s.pzt[1];
  s.px[1] = s.px[2]; s.py[1] = s.py[2]; s.pzt[1] = s.pzt[2];
  s.px[2] = x; s.py[2] = y; s.pzt[2] = z;
  nvert++;
}

// mjc_ConvexHField (convex.c:1173-1356): geom 2 expressed in the height field's frame, its
// support box against the field's box, then the native solver (mjc_penetration :34-68, one
// contact) against every triangular prism of the covered sub-grid; each contact's normal is
// fixed by mjc_fixNormal and it goes to emit as it is made (the reference fixes the normals
// after the loop; each depends on its own contact only). The warm starts of geom 2 carry over
// from the support-box calls through every prism, as in the reference's single mjCCDObj.
template <int S, class Emit>
MJH_HD void colConvexHField(const mjhipModel& m, const Lane<S>& d, int g1, int g2,
                            double margin, int* status, Emit&& emit) {
  double pos1[3], mat1[9], gp2[3], gm2[9];
  for (int k = 0; k < 3; k++) { pos1[k] = d.gxpos[3*g1 + k]; gp2[k] = d.gxpos[3*g2 + k]; }
  for (int k = 0; k < 9; k++) { mat1[k] = d.geom_xmat[9*g1 + k]; gm2[k] = d.geom_xmat[9*g2 + k]; }
  const int hid = m.geom_dataid[g1];
  const int nrow = m.hfield_nrow[hid], ncol = m.hfield_ncol[hid];
  const float* data = m.hfield_data + m.hfield_adr[hid];
  const double* size1 = m.hfield_size + 4*hid;
  double vec[3], pos[3];
  sub3(vec, gp2, pos1);
  // mju_mulMatTVec (engine_util_blas.c): rows accumulated in order, zero entries skipped
  pos[0] = pos[1] = pos[2] = 0;
  for (int i = 0; i < 3; i++) {
    if (vec[i] != 0) {
      for (int j = 0; j < 3; j++) pos[j] += mat1[3*i + j]*vec[i];
    }
  }
  const double r2 = m.geom_rbound[g2];
  for (int i = 0; i < 2; i++) {
    if ((size1[i] < pos[i] - r2 - margin) || (-size1[i] > pos[i] + r2 + margin)) return;
  }
  if (size1[2] < pos[2] - r2 - margin) return;
  if (-size1[3] > pos[2] + r2 + margin) return;
  CcdShape B;
  B.kind = B.gtype = m.geom_type[g2];
  copy3(B.pos, pos);
  for (int i = 0; i < 3; i++) {                // mju_mulMatTMat3(mat, mat1, mat2)
    for (int j = 0; j < 3; j++) {
      B.mat[3*i + j] = mat1[i]*gm2[j] + mat1[3 + i]*gm2[3 + j] + mat1[6 + i]*gm2[6 + j];
    }
  }
  for (int k = 0; k < 3; k++) B.size[k] = m.geom_size[3*g2 + k];
  B.margin = 0;
  ccdMeshData(B, m, g2);
  double sv[3];
  const double ax[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
  ccdSupportLib(sv, B, ax[0]); const double xmax = sv[0];
  ccdSupportLib(sv, B, ax[1]); const double xmin = sv[0];
  ccdSupportLib(sv, B, ax[2]); const double ymax = sv[1];
  ccdSupportLib(sv, B, ax[3]); const double ymin = sv[1];
  ccdSupportLib(sv, B, ax[4]); const double zmax = sv[2];
  ccdSupportLib(sv, B, ax[5]); const double zmin = sv[2];
  if ((xmin - margin > size1[0]) || (xmax + margin < -size1[0]) ||
      (ymin - margin > size1[1]) || (ymax + margin < -size1[1]) ||
      (zmin - margin > size1[2]) || (zmax + margin < -size1[3])) {
    return;
  }
  int cmin = (int)floor((xmin + size1[0]) / (2*size1[0]) * (ncol - 1));
  int cmax = (int)ceil((xmax + size1[0]) / (2*size1[0]) * (ncol - 1));
  int rmin = (int)floor((ymin + size1[1]) / (2*size1[1]) * (nrow - 1));
  int rmax = (int)ceil((ymax + size1[1]) / (2*size1[1]) * (nrow - 1));
  cmin = cmin > 0 ? cmin : 0;
  cmax = cmax < ncol - 1 ? cmax : ncol - 1;
  rmin = rmin > 0 ? rmin : 0;
  rmax = rmax < nrow - 1 ? rmax : nrow - 1;
  B.margin = margin;
  CcdShape A;
  A.kind = A.gtype = mjhipGEOM_HFIELD;
  A.margin = 0;
  A.vert = nullptr;
  A.graph = nullptr;
  A.nvert = 0;
  A.vertindex = A.meshindex = -1;
  for (int k = 0; k < 3; k++) { A.px[k] = A.py[k] = A.pzt[k] = 0; A.pos[k] = 0; A.size[k] = 0; }
  A.pzb = -size1[3];
  const double dx = (2.0*size1[0]) / (ncol - 1), dy = (2.0*size1[1]) / (nrow - 1);
  const int N = m.opt.ccd_iterations;
  CcdMem<1> M{{d.ccdx}, {d.ccdxi}, 5 + N, mjh_ccdFaceCap(&m)};
  int cnt = 0;
  for (int r = rmin; r < rmax; r++) {
    int nvert = 0;
    for (int c = cmin; c <= cmax; c++) {
      for (int i = 0; i < 2; i++) {
        const int rr = r + (i == 0 ? 1 : 0);
        prismAddVert(nvert, A, dx*c - size1[0], dy*rr - size1[1],
                     (double)data[rr*ncol + c]*size1[2] + margin);
        if (nvert <= 2) continue;
        if (A.pzt[0] < zmin && A.pzt[1] < zmin && A.pzt[2] < zmin) continue;
        CcdState st;
        const double dist = ccdRun(st, M, A, B, N, m.opt.ccd_tolerance, 0.0);
        if (st.unsupported) {
          *status |= MJHIP_INST_UNSUPPORTED;
          return;
        }
        if (!(dist < 0)) continue;
        double dir[3], vp[3];
        sub3(dir, st.x1, st.x2);
        normalize3(dir);
        vp[0] = 0.5*(st.x1[0] + st.x2[0]);
        vp[1] = 0.5*(st.x1[1] + st.x2[1]);
        vp[2] = 0.5*(st.x1[2] + st.x2[2]);
        RawContact con;
        con.dist = dist;
        mulMatVec3(con.frame, mat1, dir);
        mulMatVec3(con.pos, mat1, vp);
        addTo3(con.pos, pos1);
        for (int k = 3; k < 9; k++) con.frame[k] = 0;
        fixNormal(m, d, con, g1, g2);
        if (!emit(con)) return;
        if (++cnt >= 50) return;
      }
    }
  }
}
#if defined(__clang__)
#if defined(MJH_CONTRACT_OFF)
#pragma clang fp contract(off)           // a unit compiled without contraction throughout
#else
#pragma clang fp contract(fast)          // the default of this build again (see above)
#endif
#endif

// mj_collideGeoms (engine_collision_driver.c:1440-1620) + mj_setContact (:1387-1415)
// WRITE = false only counts the contacts the pair produces (the cooperative constraint
// kernel's first pass: it needs each pair's count to place the contacts in order)
// bbuf: per-lane room for box-box positions (24 x 3 doubles), or nullptr to use the
// contact list's free tail at ncon (the capacity holds 24 contacts for every box pair)
struct ContactParam;
template <int S, bool WRITE = true, bool BOX = true, bool CONVEX = true>
MJH_HD void collidePlaneBoxCyl(const mjhipModel& m, const Lane<S>& d, int g1, int g2,
                               double margin, const ContactParam& cp, int& ncon, int* status,
                               double* bbuf = nullptr);

// the narrowphase of a type-ordered primitive pair past the filters (mj_collideGeoms' call of
// mjCOLLISIONFUNC, engine_collision_driver.c:1500-1510): its raw contacts (<= 2) in raw. The
// frames may live in the mirror (SP) or in LDS (plain pointers).
template <class P, class M>
MJH_HD int narrowPrimitive(int t1, int t2, double margin, P pos1, M mat1, const double* size1,
                           P pos2, M mat2, const double* size2, RawContact raw[2]) {
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_ELLIPSOID) {
    return colPlaneEllipsoid(raw[0], margin, pos1, mat1, pos2, mat2, size2);
  }
  int num = 0;
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_SPHERE) {
    num = rawPlaneSphere(raw, margin, pos1, mat1, pos2, size2[0]);
  } else if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_CAPSULE) {
    num = colPlaneCapsule(raw, margin, pos1, mat1, pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_SPHERE) {
    num = rawSphereSphere(raw, margin, pos1, mat1, size1[0], pos2, mat2, size2[0]);
  } else if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_CAPSULE) {
    num = colSphereCapsule(raw, margin, pos1, mat1, size1[0], pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_CYLINDER) {
    num = colSphereCylinder(raw, margin, pos1, mat1, size1[0], pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_CAPSULE && t2 == mjhipGEOM_BOX) {
    num = colCapsuleBox(raw, margin, pos1, mat1, size1, pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_BOX) {
    num = rawSphereBox(raw, margin, pos1, size1[0], pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_CAPSULE && t2 == mjhipGEOM_CAPSULE) {
    num = colCapsuleCapsule(raw, margin, pos1, mat1, size1, pos2, mat2, size2);
  }
  return num;
}

// mj_collideGeoms up to the narrowphase: type-orders (g1, g2), applies the static and
// bounding-sphere filters and returns the raw contacts of a primitive or convex pair in raw
// (<= 2, with the pair's margin), 0 for none, or -1 for plane : box / cylinder, whose contacts
// collidePlaneBoxCyl stores as it makes them. CONVEX = false (the cooperative kernel, which
// no model with a convex pair launches) compiles the GJK/EPA path out.
// A predefined pair (ipair >= 0, its geoms in g1, g2) skips the bitmask filter and takes the
// pair's margin (mj_collideGeoms :1445-1492).
template <int S, bool CONVEX = true>
MJH_HD int narrowGeoms(const mjhipModel& m, const Lane<S>& d, int& g1, int& g2,
                       double& margin, RawContact raw[2], int* status, int ipair = -1) {
  if (m.geom_type[g1] > m.geom_type[g2]) { int t = g1; g1 = g2; g2 = t; }
  int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
  const int kmax = mjhip_pairMaxContacts(&m, t1, t2);
  if (kmax == 0) return 0;
  if (ipair < 0 && mjhip_filterBitmask(m.geom_contype[g1], m.geom_conaffinity[g1],
                                       m.geom_contype[g2], m.geom_conaffinity[g2])) {
    return 0;
  }
  const int ovr = (m.opt.enableflags & mjhipENBL_OVERRIDE) != 0;
  margin = ovr ? m.opt.o_margin : ipair >= 0 ? m.pair_margin[ipair] :
           (m.geom_margin[g1] > m.geom_margin[g2] ? m.geom_margin[g1] : m.geom_margin[g2]);
  if (filterSphere(m, d, g1, g2, margin)) return 0;
  if (kmax < 0) {                       // the reference would run a function not built here
    *status |= MJHIP_INST_UNSUPPORTED;
    return 0;
  }
  if (t1 == mjhipGEOM_PLANE && (t2 == mjhipGEOM_BOX || t2 == mjhipGEOM_CYLINDER)) return -1;
  if (t1 == mjhipGEOM_BOX && t2 == mjhipGEOM_BOX) return -1;
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_MESH) return -1;   // up to 3, stored as made
  if (t1 == mjhipGEOM_HFIELD) return -1;                            // up to 50, stored as made
  if (CONVEX && multiCcdPair(m, t1, t2)) return -1;                 // up to 5, stored as made
  SP<S> pos1 = d.gxpos + 3*g1, mat1 = d.geom_xmat + 9*g1;
  SP<S> pos2 = d.gxpos + 3*g2, mat2 = d.geom_xmat + 9*g2;
  const double *size1 = m.geom_size + 3*g1, *size2 = m.geom_size + 3*g2;
  if (mjhip_isConvexPair(t1, t2)) {
    if constexpr (CONVEX) {
      return colConvex(raw[0], m, d, g1, g2, margin, status);
    } else {
      *status |= MJHIP_INST_UNSUPPORTED;   // not reached: such models use one lane each
      return 0;
    }
  }
  return narrowPrimitive(t1, t2, margin, pos1, mat1, size1, pos2, mat2, size2, raw);
}

// a geom pair's contact parameters (mj_contactParam, engine_collision_driver.c:1326-1384):
// model constants, so the cooperative kernel's pair program carries them precomputed
struct ContactParam {
  int condim;
  double gap, solref[2], solimp[5], friction[5];
  double solreffriction[2];            // a predefined pair's, else 0 (mj_collideGeoms :1443)
};

// the contact parameters of geoms g1, g2: a predefined pair's own (mj_collideGeoms
// :1597-1609: solreffriction only when one of its two values is nonzero), else
// mj_contactParam's mix of the two geoms'
MJH_HD void pairParam(const mjhipModel& m, int g1, int g2, int ipair, ContactParam& cp) {
  cp.solreffriction[0] = cp.solreffriction[1] = 0;
  if (ipair < 0) {
    contactParam(m, g1, g2, &cp.condim, &cp.gap, cp.solref, cp.solimp, cp.friction);
    return;
  }
  cp.condim = m.pair_dim[ipair];
  cp.gap = m.pair_gap[ipair];
  for (int i = 0; i < 2; i++) cp.solref[i] = m.pair_solref[2*ipair + i];
  for (int i = 0; i < 5; i++) cp.solimp[i] = m.pair_solimp[5*ipair + i];
  for (int i = 0; i < 5; i++) cp.friction[i] = m.pair_friction[5*ipair + i];
  const double* sf = m.pair_solreffriction + 2*ipair;
  if (sf[0] || sf[1]) {
    cp.solreffriction[0] = sf[0];
    cp.solreffriction[1] = sf[1];
  }
}

// mj_setContact (:1387-1415) for a primitive pair's raw contacts at contact index ncon on,
// with the pair's parameters
template <int S>
MJH_HD void storeContacts(const mjhipModel& m, const Lane<S>& d, int g1, int g2, double margin,
                          const ContactParam& cp, const RawContact raw[2], int num, int& ncon,
                          int* status) {
  const int ovr = (m.opt.enableflags & mjhipENBL_OVERRIDE) != 0;
  // one raw contact into the contact list (mj_setContact); false when the list is full
  auto store = [&](const RawContact& rk) MJH_LAMBDA_INLINE -> bool {
    int i = ncon;
    if (i >= d.con_cap) {              // mjWARN_CONTACTFULL analogue (capacity is exact)
      *status |= MJHIP_INST_CNSTRFULL;
      return false;
    }
    double frame[9];
    for (int j = 0; j < 9; j++) frame[j] = rk.frame[j];
    d.con_dist[i] = rk.dist;
    copy3(d.con_pos + 3*i, rk.pos);
    d.con_geom[2*i] = g1;
    d.con_geom[2*i+1] = g2;
    d.con_dim[i] = cp.condim;
    double includemargin = margin - cp.gap;
    d.con_includemargin[i] = includemargin;
    for (int j = 0; j < 2; j++) d.con_solref[2*i+j] = ovr ? m.opt.o_solref[j] : cp.solref[j];
    for (int j = 0; j < 2; j++) {
      d.con_solreffriction[2*i+j] = ovr ? m.opt.o_solref[j] : cp.solreffriction[j];
    }
    for (int j = 0; j < 5; j++) d.con_solimp[5*i+j] = ovr ? m.opt.o_solimp[j] : cp.solimp[j];
    for (int j = 0; j < 5; j++) {
      double f = ovr ? m.opt.o_friction[j] : cp.friction[j];
      d.con_friction[5*i+j] = f > 1e-5 ? f : 1e-5;      // mjMINMU
    }
    d.con_exclude[i] = rk.dist >= includemargin;
    makeFrame(frame);
    for (int j = 0; j < 9; j++) d.con_frame[9*i+j] = frame[j];
    d.con_efc_address[i] = -1;
    d.con_mu[i] = 0;
    ncon = i + 1;
    return true;
  };
  if (store(raw[0]) && num > 1) store(raw[1]);   // num <= 2; constant indices keep raw[]
}                                                // in registers

// mj_collideGeoms (engine_collision_driver.c:1440-1620) + mj_setContact (:1387-1415) of
// geoms g1, g2, or of predefined pair ipair (g1, g2 then its geoms)
// WRITE = false only counts the contacts the pair produces
template <int S, bool WRITE = true>
MJH_HD void collideGeoms(const mjhipModel& m, const Lane<S>& d, int g1, int g2, int& ncon,
                         int* status, int ipair = -1) {
  double margin = 0;
  RawContact raw[2];
  const int num = narrowGeoms(m, d, g1, g2, margin, raw, status, ipair);
  if (!num) return;
  if (num > 0 && !WRITE) {
    ncon += num;
    return;
  }
  ContactParam cp;
  pairParam(m, g1, g2, ipair, cp);
  if (num < 0) {
    collidePlaneBoxCyl<S, WRITE>(m, d, g1, g2, margin, cp, ncon, status);
    return;
  }
  if constexpr (WRITE) storeContacts(m, d, g1, g2, margin, cp, raw, num, ncon, status);
}

// mj_setContact (:1387-1415) of one raw contact at index ncon; false when the list is full
template <int S, bool WRITE>
MJH_HD bool putContact(const mjhipModel& m, const Lane<S>& d, int g1, int g2, double margin,
                       const ContactParam& cp, const RawContact& rk, int& ncon, int* status) {
  if constexpr (!WRITE) {
    ncon++;
    return true;
  }
  const int ovr = (m.opt.enableflags & mjhipENBL_OVERRIDE) != 0;
  int i = ncon;
  if (i >= d.con_cap) {
    *status |= MJHIP_INST_CNSTRFULL;
    return false;
  }
  double frame[9];
  for (int j = 0; j < 9; j++) frame[j] = rk.frame[j];
  d.con_dist[i] = rk.dist;
  copy3(d.con_pos + 3*i, rk.pos);
  d.con_geom[2*i] = g1;
  d.con_geom[2*i+1] = g2;
  d.con_dim[i] = cp.condim;
  double includemargin = margin - cp.gap;
  d.con_includemargin[i] = includemargin;
  for (int j = 0; j < 2; j++) d.con_solref[2*i+j] = ovr ? m.opt.o_solref[j] : cp.solref[j];
  for (int j = 0; j < 2; j++) {
    d.con_solreffriction[2*i+j] = ovr ? m.opt.o_solref[j] : cp.solreffriction[j];
  }
  for (int j = 0; j < 5; j++) d.con_solimp[5*i+j] = ovr ? m.opt.o_solimp[j] : cp.solimp[j];
  for (int j = 0; j < 5; j++) {
    double f = ovr ? m.opt.o_friction[j] : cp.friction[j];
    d.con_friction[5*i+j] = f > 1e-5 ? f : 1e-5;      // mjMINMU
  }
  d.con_exclude[i] = rk.dist >= includemargin;
  makeFrame(frame);
  for (int j = 0; j < 9; j++) d.con_frame[9*i+j] = frame[j];
  d.con_efc_address[i] = -1;
  d.con_mu[i] = 0;
  ncon = i + 1;
  return true;
}

// box : box (up to 24 raw contacts)
template <int S, bool WRITE>
MJH_HD void collideBoxBox(const mjhipModel& m, const Lane<S>& d, int g1, int g2,
                          double margin, const ContactParam& cp, int& ncon, int* status,
                          double* bbuf) {
  double p1[3], m1[9], p2[3], m2[9];
  for (int k = 0; k < 3; k++) { p1[k] = d.gxpos[3*g1 + k]; p2[k] = d.gxpos[3*g2 + k]; }
  for (int k = 0; k < 9; k++) { m1[k] = d.geom_xmat[9*g1 + k]; m2[k] = d.geom_xmat[9*g2 + k]; }
  const double *size1 = m.geom_size + 3*g1, *size2 = m.geom_size + 3*g2;
  unsigned keep;
  if (bbuf) {
    keep = boxBoxKeep(margin, p1, m1, size1, p2, m2, size2, bbuf);
  } else {
    // the exact capacity holds 24 contacts for every box pair, so this is reached only in a
    // capped context (mjhip_contextCreateCapped): the instance is flagged CNSTRFULL and the
    // pair is dropped whole, as the reference drops a pair whose mjContact[mjMAXCONPAIR]
    // scratch does not fit in the arena (mj_collideGeoms, engine_collision_driver.c:1499-1505,
    // mjWARN_CONTACTFULL). The threshold differs: the reference's is the arena's free bytes
    // for 50 contacts, ours the list's tail for this path's 24 (its scratch)
    if (ncon + 24 > d.con_cap) {
      *status |= MJHIP_INST_CNSTRFULL;
      return;
    }
    keep = boxBoxKeep(margin, p1, m1, size1, p2, m2, size2, d.con_pos + 3*ncon);
  }
  bool ok = true;
  boxBoxEmit(margin, p1, m1, size1, p2, m2, size2, keep,
             [&](const RawContact& rk) MJH_LAMBDA_INLINE {
    if (ok) ok = putContact<S, WRITE>(m, d, g1, g2, margin, cp, rk, ncon, status);
  });
}

// plane : box / cylinder (up to 4 contacts each), box : box (up to 24), plane : mesh (up to
// 3) and height field : geom (up to 50): contacts are stored as they are made. BOX = false
// compiles the box-box path out (kernels launched for models without a box pair: its private
// arrays would otherwise cost every contact kernel); CONVEX = false compiles the mesh and
// height-field paths out (the cooperative kernel, which no such model launches)
template <int S, bool WRITE, bool BOX, bool CONVEX>
MJH_HD void collidePlaneBoxCyl(const mjhipModel& m, const Lane<S>& d, int g1, int g2,
                               double margin, const ContactParam& cp, int& ncon, int* status,
                               double* bbuf) {
  if (multiCcdPair(m, m.geom_type[g1], m.geom_type[g2])) {     // before box-box: box-mesh
    if constexpr (CONVEX) {
      colConvexMulti(m, d, g1, g2, margin, status,
                     [&](const RawContact& rk) MJH_LAMBDA_INLINE -> bool {
        return putContact<S, WRITE>(m, d, g1, g2, margin, cp, rk, ncon, status);
      });
    } else {
      *status |= MJHIP_INST_UNSUPPORTED;      // not reached: such models use one lane each
    }
    return;
  }
  if (m.geom_type[g1] == mjhipGEOM_BOX) {
    if constexpr (BOX) collideBoxBox<S, WRITE>(m, d, g1, g2, margin, cp, ncon, status, bbuf);
    else *status |= MJHIP_INST_UNSUPPORTED;   // not reached: the launch saw no box pair
    return;
  }
  if (m.geom_type[g1] == mjhipGEOM_HFIELD || m.geom_type[g2] == mjhipGEOM_MESH) {
    if constexpr (CONVEX) {
      auto store = [&](const RawContact& rk) MJH_LAMBDA_INLINE -> bool {
        return putContact<S, WRITE>(m, d, g1, g2, margin, cp, rk, ncon, status);
      };
      if (m.geom_type[g1] == mjhipGEOM_HFIELD) {
        colConvexHField(m, d, g1, g2, margin, status, store);
      } else {
        colPlaneMesh(m, d, g1, g2, margin, store);
      }
    } else {
      *status |= MJHIP_INST_UNSUPPORTED;      // not reached: such models use one lane each
    }
    return;
  }
  SP<S> pos1 = d.gxpos + 3*g1, mat1 = d.geom_xmat + 9*g1;
  SP<S> pos2 = d.gxpos + 3*g2, mat2 = d.geom_xmat + 9*g2;
  const double* size2 = m.geom_size + 3*g2;
  auto store = [&](const RawContact& rk) MJH_LAMBDA_INLINE -> bool {
    return putContact<S, WRITE>(m, d, g1, g2, margin, cp, rk, ncon, status);
  };
  if (m.geom_type[g2] == mjhipGEOM_BOX) {
    colPlaneBox(margin, pos1, mat1, pos2, mat2, size2, store);
  } else {
    colPlaneCylinder(margin, pos1, mat1, pos2, mat2, size2, store);
  }
}

// engine_support.c:1407-1450 mj_geomDistance (the oracle's or_geomDistance): the smallest
// signed distance between two geoms up to distmax and the segment between the nearest
// points (zeros when none is found); mjc_Convex and box-box pairs through the native solver
// with the bound as its cutoff (mj_geomDistanceCCD :1379-1402), the rest through their
// collision functions with the bound as the margin. Functions outside the subset flag.
template <int S>
MJH_HD double geomDistance(const mjhipModel& m, const Lane<S>& d, int geom1, int geom2,
                           double distmax, double fromto[6], int* status) {
  double dist = distmax;
  for (int k = 0; k < 6; k++) fromto[k] = 0;
  const bool flip = m.geom_type[geom1] > m.geom_type[geom2];
  const int g1 = flip ? geom2 : geom1, g2 = flip ? geom1 : geom2;
  const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
  const bool nccd = !(m.opt.disableflags & mjhipDSBL_NATIVECCD);
  const bool ccd = nccd && (mjhip_isConvexPair(t1, t2) ||
                            (t1 == mjhipGEOM_BOX && t2 == mjhipGEOM_BOX));
  const int kmax = mjhip_pairMaxContacts(&m, t1, t2);
  if (kmax == 0) return dist;
  if ((kmax < 0 && !ccd) || (t1 == mjhipGEOM_BOX && t2 == mjhipGEOM_BOX && !ccd)) {
    *status |= MJHIP_INST_UNSUPPORTED;   // refused at context creation (mjhip.hip)
    return dist;
  }
  if (ccd) {
    const int N = m.opt.ccd_iterations;
    CcdMem<1> M{{d.ccdx}, {d.ccdxi}, 5 + N, mjh_ccdFaceCap(&m)};
    CcdShape A, B;
    ccdShape(A, m, d, g1, 0.0);
    ccdShape(B, m, d, g2, 0.0);
    CcdState st;
    const double r = ccdRun(st, M, A, B, N, m.opt.ccd_tolerance, distmax);
    if (st.unsupported) *status |= MJHIP_INST_UNSUPPORTED;
    if (st.nx > 0) {
      for (int k = 0; k < 3; k++) fromto[k] = st.x1[k];
      for (int k = 0; k < 3; k++) fromto[3+k] = st.x2[k];
    }
    return r;
  }
  double pos1[3], mat1[9], pos2[3], mat2[9];
  for (int k = 0; k < 3; k++) { pos1[k] = d.geom_xpos[3*g1+k]; pos2[k] = d.geom_xpos[3*g2+k]; }
  for (int k = 0; k < 9; k++) { mat1[k] = d.geom_xmat[9*g1+k]; mat2[k] = d.geom_xmat[9*g2+k]; }
  const double *size1 = m.geom_size + 3*g1, *size2 = m.geom_size + 3*g2;
  RawContact best;
  bool found = false;
  auto take = [&](const RawContact& rk) MJH_LAMBDA_INLINE -> bool {
    if (rk.dist < dist) {
      dist = rk.dist;
      best = rk;
      found = true;
    }
    return true;
  };
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_MESH) {
    colPlaneMesh(m, d, g1, g2, distmax, take);
  } else if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_BOX) {
    colPlaneBox(distmax, (const double*)pos1, (const double*)mat1, (const double*)pos2,
                (const double*)mat2, size2, take);
  } else if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_CYLINDER) {
    colPlaneCylinder(distmax, (const double*)pos1, (const double*)mat1, (const double*)pos2,
                     (const double*)mat2, size2, take);
  } else {
    RawContact raw[2];
    const int num = narrowPrimitive(t1, t2, distmax, (const double*)pos1, (const double*)mat1,
                                    size1, (const double*)pos2, (const double*)mat2, size2, raw);
    if (num > 0) take(raw[0]);             // constant indices keep raw[] in registers
    if (num > 1) take(raw[1]);
  }
  if (found) {
    const double sign = flip ? -1 : 1;
    for (int k = 0; k < 3; k++) {
      fromto[k] = best.pos[k] + best.frame[k]*(-0.5*sign*dist);
      fromto[3+k] = best.pos[k] + best.frame[k]*(0.5*sign*dist);
    }
  }
  return dist;
}

// mj_filterSphere (engine_collision_driver.c:1470-1497) of a program entry: 1 = the bounding
// spheres (filt 0, bound rb1 + rb2 + margin) or the plane distance (filt 1/2: plane g1/g2,
// bound margin + rb of the other geom) rule the pair out; filt 3: no test
template <int S>
MJH_HD bool programFilter(const Lane<S>& d, const CoopPair& P) {
  SP<S> p1 = d.gxpos + 3*P.g1, p2 = d.gxpos + 3*P.g2;
  if (P.filt == 0) {
    const double dif[3] = {p1[0]-p2[0], p1[1]-p2[1], p1[2]-p2[2]};
    return dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2] > P.bound*P.bound;
  }
  if (P.filt <= 2) {
    const bool pl1 = P.filt == 1;
    SP<S> mat = d.geom_xmat + 9*(pl1 ? P.g1 : P.g2);
    const double norm[3] = {mat[2], mat[5], mat[8]};
    double dif[3];
    sub3(dif, pl1 ? p2 : p1, pl1 ? p1 : p2);
    return dot3(dif, norm) > P.bound;
  }
  return false;
}

// mj_collision (engine_collision_driver.c:265-497) over the static collision program
// (csrc/pair_program.h, built once per context): the candidate body pairs in signature order,
// their geom pairs all-to-all (a midphase pair's stably sorted by contactcompare's key, as
// mj_collideTree's callers sort its contacts), and the predefined pairs merged in ahead of the
// first body pair whose signature is not below theirs (:316-327), the rest after the sweep
// (:432-437), a swept geom pair that is a predefined pair left to it (:499-523).
template <int S>
MJH_HD void collision(const mjhipModel& m, const Lane<S>& d, int* status) {
  int ncon = 0;                        // in a register; written once at the end
  d.con_count[0] = 0;
  if (!mjhip_contactsEnabled(&m)) return;
  if (d.gstage) {                      // 16 loads in flight per step
    const int n = 3*m.ngeom;
    for (int k = 0; k < n; k += 16) {
      double t[16];
#pragma unroll
      for (int i = 0; i < 16; i++) t[i] = k + i < n ? d.geom_xpos[k+i] : 0.0;
#pragma unroll
      for (int i = 0; i < 16; i++) {
        if (k + i < n) d.gxpos[k+i] = t[i];
      }
    }
  }
  // the static program (csrc/pair_program.h; nullptr when it is empty: no geom pair of the
  // model can collide): its bounding-sphere tests eight entries at a time (their position
  // loads in flight together), then the narrowphase of the survivors in program order. The
  // filter is mj_filterSphere's test with the entry's bound formed as the reference forms it,
  // so the entries it drops are the ones collideGeoms would return no contact for.
  const int np = d.prog ? d.nprog : 0;
  for (int p0 = 0; p0 < np; p0 += 8) {
    bool hit[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      hit[u] = false;
      if (p0 + u < np) hit[u] = !programFilter(d, d.prog[p0 + u]);
    }
    for (int u = 0; u < 8 && p0 + u < np; u++) {
      if (!hit[u]) continue;
      const CoopPair& P = d.prog[p0 + u];
      collideGeoms(m, d, P.g1, P.g2, ncon, status, d.prog_ipair[p0 + u]);
    }
  }
  d.con_count[0] = ncon;
}

// mj_applyFT :1194-1251 (dense)
template <int S, class F, class T, class P>
MJH_HD void applyFT(const mjhipModel& m, const Lane<S>& d, F force, T torque, P point, int body,
                    SP<S> qfrc_target) {
  jac(m, d, point, body);
  mulMatTVec(d.qforce, d.jacp, force, 3, m.nv);
  addTo(qfrc_target, d.qforce, m.nv);
  mulMatTVec(d.qforce, d.jacr, torque, 3, m.nv);
  addTo(qfrc_target, d.qforce, m.nv);
}

// torque = 0, as mj_gravcomp passes it
template <int S, class F, class P>
MJH_HD void applyForce(const mjhipModel& m, const Lane<S>& d, F force, P point, int body,
                       SP<S> qfrc_target) {
  double zt[3] = {0, 0, 0};
  applyFT(m, d, force, zt, point, body, qfrc_target);
}

//---------------------------------- engine_core_smooth.c -------------------------------------

// mj_kinematics :38-178
template <int S>
MJH_HD void kinematics(const mjhipModel& m, const Lane<S>& d) {
  int nbody = m.nbody;
  zero3(d.xpos);
  d.xquat[0] = 1; d.xquat[1] = 0; d.xquat[2] = 0; d.xquat[3] = 0;
  zero3(d.xipos);
  zero(d.xmat, 9);
  zero(d.ximat, 9);
  d.xmat[0] = 1; d.xmat[4] = 1; d.xmat[8] = 1;
  d.ximat[0] = 1; d.ximat[4] = 1; d.ximat[8] = 1;

  for (int i = 1; i < nbody; i++) {
    double xpos[3], xquat[4];
    int jntadr = m.body_jntadr[i];
    int jntnum = m.body_jntnum[i];
    if (jntnum == 1 && m.jnt_type[jntadr] == mjhipJNT_FREE) {
      int qadr = m.jnt_qposadr[jntadr];
      copy3(xpos, d.qpos + qadr);
      copy4(xquat, d.qpos + qadr + 3);
      normalize4(xquat);
      copy3(d.xanchor + 3*jntadr, xpos);
      copy3(d.xaxis + 3*jntadr, m.jnt_axis + 3*jntadr);
    } else {
      int pid = m.body_parentid[i];
      double bodypos[3], bodyquat[4];
      const int mid = m.body_mocapid[i];
      if (mid >= 0) {               // mocap body: pose from mjData (normalized quaternion)
        copy3(bodypos, d.mocap_pos + 3*mid);
        copy4(bodyquat, d.mocap_quat + 4*mid);
        normalize4(bodyquat);
      } else {
        copy3(bodypos, m.body_pos + 3*i);
        copy4(bodyquat, m.body_quat + 4*i);
      }
      if (pid) {
        mulMatVec3(xpos, d.xmat + 9*pid, bodypos);
        addTo3(xpos, d.xpos + 3*pid);
        mulQuat(xquat, d.xquat + 4*pid, bodyquat);
      } else {
        copy3(xpos, bodypos);
        copy4(xquat, bodyquat);
      }
      double xanchor[3], xaxis[3];
      for (int j = 0; j < jntnum; j++) {
        int jid = jntadr + j;
        int qadr = m.jnt_qposadr[jid];
        int jtype = m.jnt_type[jid];
        rotVecQuat(xaxis, m.jnt_axis + 3*jid, xquat);
        rotVecQuat(xanchor, m.jnt_pos + 3*jid, xquat);
        addTo3(xanchor, xpos);
        if (jtype == mjhipJNT_SLIDE) {
          addToScl3(xpos, xaxis, d.qpos[qadr] - m.qpos0[qadr]);
        } else {
          double qloc[4];
          if (jtype == mjhipJNT_BALL) {
            copy4(qloc, d.qpos + qadr);
            normalize4(qloc);
          } else {
            axisAngle2Quat(qloc, m.jnt_axis + 3*jid, d.qpos[qadr] - m.qpos0[qadr]);
          }
          mulQuat(xquat, xquat, qloc);
          double vec[3];
          rotVecQuat(vec, m.jnt_pos + 3*jid, xquat);
          sub3(xpos, xanchor, vec);
        }
        copy3(d.xanchor + 3*jid, xanchor);
        copy3(d.xaxis + 3*jid, xaxis);
      }
    }
    normalize4(xquat);
    copy4(d.xquat + 4*i, xquat);
    copy3(d.xpos + 3*i, xpos);
    quat2Mat(d.xmat + 9*i, xquat);
  }
  for (int i = 1; i < nbody; i++) {
    local2Global(d, d.xipos + 3*i, d.ximat + 9*i, m.body_ipos + 3*i, m.body_iquat + 4*i, i,
                 m.body_sameframe[i]);
  }
  for (int i = 0; i < m.ngeom; i++) {
    local2Global(d, d.geom_xpos + 3*i, d.geom_xmat + 9*i, m.geom_pos + 3*i,
                 m.geom_quat + 4*i, m.geom_bodyid[i], m.geom_sameframe[i]);
  }
  for (int i = 0; i < m.nsite; i++) {
    local2Global(d, d.site_xpos + 3*i, d.site_xmat + 9*i, m.site_pos + 3*i,
                 m.site_quat + 4*i, m.site_bodyid[i], m.site_sameframe[i]);
  }
}

// mj_comPos :183-270
template <int S>
MJH_HD void comPos(const mjhipModel& m, const Lane<S>& d) {
  int nbody = m.nbody, njnt = m.njnt;
  double offset[3], axis[3];
  SP<S> mass_subtree = d.mass_subtree;
  zero(mass_subtree, nbody);
  zero(d.subtree_com, nbody*3);
  for (int i = nbody-1; i >= 0; i--) {
    addToScl3(d.subtree_com + 3*i, d.xipos + 3*i, m.body_mass[i]);
    mass_subtree[i] += m.body_mass[i];
    if (i) {
      int j = m.body_parentid[i];
      addTo3(d.subtree_com + 3*j, d.subtree_com + 3*i);
      mass_subtree[j] += mass_subtree[i];
    }
    if (mass_subtree[i] < MINVAL) {
      copy3(d.subtree_com + 3*i, d.xipos + 3*i);
    } else {
      double ms = mass_subtree[i];
      scl3(d.subtree_com + 3*i, d.subtree_com + 3*i, 1.0/(ms > MINVAL ? ms : MINVAL));
    }
  }
  zero(d.cinert, 10);
  for (int i = 1; i < nbody; i++) {
    sub3(offset, d.xipos + 3*i, d.subtree_com + 3*m.body_rootid[i]);
    inertCom(d.cinert + 10*i, m.body_inertia + 3*i, d.ximat + 9*i, offset, m.body_mass[i]);
  }
  for (int j = 0; j < njnt; j++) {
    int da = 6*m.jnt_dofadr[j];
    int bi = m.jnt_bodyid[j];
    sub3(offset, d.subtree_com + 3*m.body_rootid[bi], d.xanchor + 3*j);
    int skip = 0;
    switch (m.jnt_type[j]) {
    case mjhipJNT_FREE:
      zero(d.cdof + da, 18);
      for (int i = 0; i < 3; i++) d.cdof[da+3+7*i] = 1;
      skip = 18;
      // fallthrough
    case mjhipJNT_BALL:
      for (int i = 0; i < 3; i++) {
        axis[0] = d.xmat[9*bi+i+0];
        axis[1] = d.xmat[9*bi+i+3];
        axis[2] = d.xmat[9*bi+i+6];
        dofComHinge(d.cdof + da + skip + 6*i, axis, offset);
      }
      break;
    case mjhipJNT_SLIDE:
      zero3(d.cdof + da);
      copy3(d.cdof + da + 3, d.xaxis + 3*j);
      break;
    case mjhipJNT_HINGE:
      dofComHinge(d.cdof + da, d.xaxis + 3*j, offset);
      break;
    }
  }
}

// mj_camlight :275-392
template <int S>
MJH_HD void camlight(const mjhipModel& m, const Lane<S>& d) {
  double pos[3], matT[9];
  for (int i = 0; i < m.ncam; i++) {
    local2Global(d, d.cam_xpos + 3*i, d.cam_xmat + 9*i, m.cam_pos + 3*i, m.cam_quat + 4*i,
                 m.cam_bodyid[i], 0);
    int id = m.cam_bodyid[i];
    int id1 = m.cam_targetbodyid[i];
    switch (m.cam_mode[i]) {
    case mjhipCAMLIGHT_TRACK:
    case mjhipCAMLIGHT_TRACKCOM:
      copy(d.cam_xmat + 9*i, m.cam_mat0 + 9*i, 9);
      if (m.cam_mode[i] == mjhipCAMLIGHT_TRACK) {
        add3(d.cam_xpos + 3*i, d.xpos + 3*id, m.cam_pos0 + 3*i);
      } else {
        add3(d.cam_xpos + 3*i, d.subtree_com + 3*id, m.cam_poscom0 + 3*i);
      }
      break;
    case mjhipCAMLIGHT_TARGETBODY:
    case mjhipCAMLIGHT_TARGETBODYCOM:
      if (id1 >= 0) {
        if (m.cam_mode[i] == mjhipCAMLIGHT_TARGETBODY) {
          copy3(pos, d.xpos + 3*id1);
        } else {
          copy3(pos, d.subtree_com + 3*id1);
        }
        sub3(matT + 6, d.cam_xpos + 3*i, pos);
        normalize3(matT + 6);
        matT[3] = 0; matT[4] = 0; matT[5] = 1;
        cross(matT, matT + 3, matT + 6);
        normalize3(matT);
        cross(matT + 3, matT + 6, matT);
        normalize3(matT + 3);
        for (int r = 0; r < 3; r++)
          for (int c = 0; c < 3; c++) d.cam_xmat[9*i + 3*c + r] = matT[3*r + c];
      }
      break;
    default:
      break;
    }
  }
  for (int i = 0; i < m.nlight; i++) {
    int id = m.light_bodyid[i];
    int id1 = m.light_targetbodyid[i];
    // mj_local2Global with xmat = 0 (position only)
    mulMatVec3(d.light_xpos + 3*i, d.xmat + 9*id, m.light_pos + 3*i);
    addTo3(d.light_xpos + 3*i, d.xpos + 3*id);
    rotVecQuat(d.light_xdir + 3*i, m.light_dir + 3*i, d.xquat + 4*id);
    switch (m.light_mode[i]) {
    case mjhipCAMLIGHT_TRACK:
    case mjhipCAMLIGHT_TRACKCOM:
      copy3(d.light_xdir + 3*i, m.light_dir0 + 3*i);
      if (m.light_mode[i] == mjhipCAMLIGHT_TRACK) {
        add3(d.light_xpos + 3*i, d.xpos + 3*id, m.light_pos0 + 3*i);
      } else {
        add3(d.light_xpos + 3*i, d.subtree_com + 3*id, m.light_poscom0 + 3*i);
      }
      break;
    case mjhipCAMLIGHT_TARGETBODY:
    case mjhipCAMLIGHT_TARGETBODYCOM:
      if (id1 >= 0) {
        if (m.light_mode[i] == mjhipCAMLIGHT_TARGETBODY) {
          copy3(pos, d.xpos + 3*id1);
        } else {
          copy3(pos, d.subtree_com + 3*id1);
        }
        sub3(d.light_xdir + 3*i, pos, d.light_xpos + 3*i);
      }
      break;
    default:
      break;
    }
    normalize3(d.light_xdir + 3*i);
  }
}

// ---- tendon wrapping around spheres and cylinders (engine_util_misc.c:33-418), on plain
// per-lane doubles
MJH_HD double dot2(const double* a, const double* b) { return 0.0 + (a[0]*b[0] + a[1]*b[1]); }

// mju_normalize, n = 2 (engine_util_blas.c:651-668)
MJH_HD double normalize2(double* v) {
  double norm = sqrt(dot2(v, v));
  if (norm < MINVAL) {
    v[0] = 1; v[1] = 0;
  } else {
    double inv = 1/norm;
    v[0] *= inv; v[1] *= inv;
  }
  return norm;
}

// :33-50 segments p1-p2 and p3-p4 intersect
MJH_HD bool wrapIntersect(const double* p1, const double* p2, const double* p3,
                          const double* p4) {
  double det = (p4[1]-p3[1])*(p2[0]-p1[0]) - (p4[0]-p3[0])*(p2[1]-p1[1]);
  if (fabs(det) < MINVAL) return false;
  double a = ((p4[0]-p3[0])*(p1[1]-p3[1]) - (p4[1]-p3[1])*(p1[0]-p3[0])) / det;
  double b = ((p2[0]-p1[0])*(p1[1]-p3[1]) - (p2[1]-p1[1])*(p1[0]-p3[0])) / det;
  return a >= 0 && a <= 1 && b >= 0 && b <= 1;
}

// :77-151 circle wrap: tangent points pnt[4] and arc length, or -1 when the segment clears
MJH_HD double wrapCircle(double pnt[4], const double end[4], const double* side,
                         double radius) {
  const double sqlen0 = end[0]*end[0] + end[1]*end[1];
  const double sqlen1 = end[2]*end[2] + end[3]*end[3];
  const double sqrad = radius*radius;
  if (sqlen0 < sqrad || sqlen1 < sqrad || radius < MINVAL) return -1;
  const double dif[2] = {end[2]-end[0], end[3]-end[1]};
  const double dd = dif[0]*dif[0] + dif[1]*dif[1];
  if (dd < MINVAL) return -1;
  double a = -(dif[0]*end[0] + dif[1]*end[1])/dd;
  a = a < 0 ? 0 : (a > 1 ? 1 : a);
  double tmp[2] = {a*dif[0] + end[0], a*dif[1] + end[1]};
  if (tmp[0]*tmp[0] + tmp[1]*tmp[1] > sqrad && (!side || dot2(side, tmp) >= 0)) return -1;
  const double sqrt0 = sqrt(sqlen0 - sqrad), sqrt1 = sqrt(sqlen1 - sqrad);
  double sol[2][4], good[2];
  for (int i = 0; i < 2; i++) {
    const int sgn = i == 0 ? 1 : -1;
    sol[i][0] = (end[0]*sqrad + sgn*radius*end[1]*sqrt0)/sqlen0;
    sol[i][1] = (end[1]*sqrad - sgn*radius*end[0]*sqrt0)/sqlen0;
    sol[i][2] = (end[2]*sqrad - sgn*radius*end[3]*sqrt1)/sqlen1;
    sol[i][3] = (end[3]*sqrad + sgn*radius*end[2]*sqrt1)/sqlen1;
    if (side) {
      tmp[0] = sol[i][0] + sol[i][2];
      tmp[1] = sol[i][1] + sol[i][3];
      normalize2(tmp);
      good[i] = dot2(tmp, side);
    } else {
      tmp[0] = sol[i][0] - sol[i][2];
      tmp[1] = sol[i][1] - sol[i][3];
      good[i] = -dot2(tmp, tmp);
    }
    if (wrapIntersect(end, sol[i], end + 2, sol[i] + 2)) good[i] = -10000;
  }
  const int i = good[0] > good[1] ? 0 : 1;
  for (int k = 0; k < 4; k++) pnt[k] = sol[i][k];
  if (wrapIntersect(end, pnt, end + 2, pnt + 2)) return -1;
  // :55-71 arc length, the long way round for the second solution's orientation
  double p0n[2] = {pnt[0], pnt[1]}, p1n[2] = {pnt[2], pnt[3]};
  normalize2(p0n);
  normalize2(p1n);
  double angle = acos(dot2(p0n, p1n));
  const double cr = pnt[1]*pnt[2] - pnt[0]*pnt[3];
  if ((cr > 0 && i) || (cr < 0 && !i)) angle = 2*mjhipPI - angle;
  return radius*angle;
}

// :157-272 inside wrap (side site within the circle): one contact point by Newton
// iterations on asin(A z) + asin(B z) - 2 asin(z) + G = 0; returns 0, or -1
MJH_HD double wrapInside(double pnt[4], const double end[4], double radius) {
  const double len0 = sqrt(dot2(end, end)), len1 = sqrt(dot2(end + 2, end + 2));
  const double dif[2] = {end[2]-end[0], end[3]-end[1]};
  const double dd = dif[0]*dif[0] + dif[1]*dif[1];
  if (len0 <= radius || len1 <= radius || radius < MINVAL || len0 < MINVAL || len1 < MINVAL) {
    return -1;
  }
  if (dd > MINVAL) {
    const double a = -(dif[0]*end[0] + dif[1]*end[1]) / dd;
    if (a > 0 && a < 1) {
      const double tmp[2] = {end[0] + a*dif[0], end[1] + a*dif[1]};
      if (sqrt(dot2(tmp, tmp)) <= radius) return -1;
    }
  }
  pnt[0] = 0.5*(end[0] + end[2]);
  pnt[1] = 0.5*(end[1] + end[3]);
  normalize2(pnt);
  pnt[0] *= radius;
  pnt[1] *= radius;
  pnt[2] = pnt[0];
  pnt[3] = pnt[1];
  const double A = radius/len0, B = radius/len1;
  const double cosG = (len0*len0 + len1*len1 - dd) / (2*len0*len1);
  if (cosG < -1 + MINVAL) return -1;
  if (cosG > 1 - MINVAL) return 0;
  const double G = acos(cosG);
  double z = 1 - 1e-7;
  double f = asin(A*z) + asin(B*z) - 2*asin(z) + G;
  if (f > 0) return 0;
  int iter;
  for (iter = 0; iter < 20 && fabs(f) > 1e-6; iter++) {
    const double df = A/fmax(MINVAL, sqrt(1 - z*z*A*A)) + B/fmax(MINVAL, sqrt(1 - z*z*B*B)) -
                      2/fmax(MINVAL, sqrt(1 - z*z));
    if (df > -MINVAL) return 0;
    const double z1 = z - f/df;
    if (z1 > z) return 0;
    z = z1;
    f = asin(A*z) + asin(B*z) - 2*asin(z) + G;
    if (f > 1e-6) return 0;
  }
  if (iter >= 20) return 0;
  double vec[2], ang;
  if (end[0]*end[3] - end[1]*end[2] > 0) {
    vec[0] = end[0]; vec[1] = end[1];
    ang = asin(z) - asin(A*z);
  } else {
    vec[0] = end[2]; vec[1] = end[3];
    ang = asin(z) - asin(B*z);
  }
  normalize2(vec);
  pnt[0] = radius*(cos(ang)*vec[0] - sin(ang)*vec[1]);
  pnt[1] = radius*(sin(ang)*vec[0] + cos(ang)*vec[1]);
  pnt[2] = pnt[0];
  pnt[3] = pnt[1];
  return 0;
}

// :282-418 mju_wrap: segment x0-x1 around the sphere/cylinder at xpos/xmat; the tangent
// points (global frame) in wpnt[6] and the wrapped length, or -1 for no wrap
MJH_HD double wrapGeom(double wpnt[6], const double x0[3], const double x1[3],
                       const double xpos[3], const double xmat[9], double radius, int type,
                       const double* side) {
  double tmp[3], p0[3], p1[3];
  sub3(tmp, x0, xpos);
  mulMatTVec3(p0, xmat, tmp);
  sub3(tmp, x1, xpos);
  mulMatTVec3(p1, xmat, tmp);
  if (sqrt(dot3(p0, p0)) < MINVAL || sqrt(dot3(p1, p1)) < MINVAL) return -1;
  double ax0[3], ax1[3];
  if (type == mjhipWRAP_SPHERE) {
    copy3(ax0, p0);
    normalize3(ax0);
    double normal[3];
    cross(normal, p0, p1);
    if (normalize3(normal) < MINVAL) {        // p0, p1 parallel: any normal
      int i = 0;
      if (fabs(ax0[1]) > fabs(ax0[0]) && fabs(ax0[1]) > fabs(ax0[2])) i = 1;
      if (fabs(ax0[2]) > fabs(ax0[0]) && fabs(ax0[2]) > fabs(ax0[1])) i = 2;
      ax1[0] = 1; ax1[1] = 1; ax1[2] = 1;
      ax1[i] = 0;
      cross(normal, ax0, ax1);
      normalize3(normal);
    }
    cross(ax1, normal, ax0);
    normalize3(ax1);
  } else {
    ax0[0] = 1; ax0[1] = 0; ax0[2] = 0;
    ax1[0] = 0; ax1[1] = 1; ax1[2] = 0;
  }
  const double end[4] = {dot3(p0, ax0), dot3(p0, ax1), dot3(p1, ax0), dot3(p1, ax1)};
  double s[3], sd[2];
  if (side) {
    sub3(tmp, side, xpos);
    mulMatTVec3(s, xmat, tmp);
    sd[0] = dot3(s, ax0);
    sd[1] = dot3(s, ax1);
    normalize2(sd);
    sd[0] *= radius;
    sd[1] *= radius;
  }
  double pnt[4];
  double wlen = side && sqrt(dot3(s, s)) < radius ? wrapInside(pnt, end, radius)
                                                  : wrapCircle(pnt, end, side ? sd : nullptr, radius);
  if (wlen < 0) return -1;
  double res[6];
  for (int i = 0; i < 2; i++) {
    scl3(res + 3*i, ax0, pnt[2*i]);
    scl3(tmp, ax1, pnt[2*i + 1]);
    addTo3(res + 3*i, tmp);
  }
  if (type == mjhipWRAP_CYLINDER) {           // spread the height change along the path
    const double L0 = sqrt((p0[0]-res[0])*(p0[0]-res[0]) + (p0[1]-res[1])*(p0[1]-res[1]));
    const double L1 = sqrt((p1[0]-res[3])*(p1[0]-res[3]) + (p1[1]-res[4])*(p1[1]-res[4]));
    res[2] = p0[2] + (p1[2] - p0[2])*L0 / (L0+wlen+L1);
    res[5] = p0[2] + (p1[2] - p0[2])*(L0+wlen) / (L0+wlen+L1);
    const double height = fabs(res[5] - res[2]);
    wlen = sqrt(wlen*wlen + height*height);
  }
  mulMatVec3(wpnt, xmat, res);
  mulMatVec3(wpnt + 3, xmat, res + 3);
  addTo3(wpnt, xpos);
  addTo3(wpnt + 3, xpos);
  return wlen;
}

// mj_tendon :651-860 (fixed tendons; spatial tendons through sites, pulleys and wrapping
// spheres/cylinders); dense ten_J, or the compressed rows of a sparse-mode model (:668-719,
// :801-819: each joint / path segment merged into the row by mju_combineSparse)
template <int S>
MJH_HD void tendon(const mjhipModel& m, const Lane<S>& d) {
  int nv = m.nv, nten = m.ntendon;
  if (!nten) return;
  const bool sparse = mjh_isSparse(&m);
  zero(d.ten_length, nten);
  if (sparse) {
    for (int i = 0; i < nten; i++) d.ten_J_rownnz[i] = 0;
  } else {
    zero(d.ten_J, nten*nv);
  }
  for (int i = 0; i < nten; i++) {
    int adr = m.tendon_adr[i];
    int num = m.tendon_num[i];
    const int radr = sparse ? (i ? d.ten_J_rowadr[i-1] + d.ten_J_rownnz[i-1] : 0) : 0;
    if (sparse) d.ten_J_rowadr[i] = radr;
    if (m.wrap_type[adr] == mjhipWRAP_JOINT) {
      for (int j = 0; j < num; j++) {
        int k = m.wrap_objid[adr+j];
        d.ten_length[i] += m.wrap_prm[adr+j] * d.qpos[m.jnt_qposadr[k]];
        if (sparse) {
          d.ten_J_rownnz[i] = combineSparse(d.ten_J + radr, m.wrap_prm + adr + j, 1.0, 1.0,
                                            d.ten_J_rownnz[i], 1, d.ten_J_colind + radr,
                                            m.jnt_dofadr + k, d.sparse_buf, d.chainbuf + 2*nv);
        } else {
          d.ten_J[i*nv + m.jnt_dofadr[k]] = m.wrap_prm[adr+j];
        }
      }
      continue;
    }
    // spatial: site-site or site-geom-site sequences; a pulley divides the length and
    // moment that follow
    double divisor = 1;
    int j = 0;
    while (j < num - 1) {
      const int type0 = m.wrap_type[adr+j], type1 = m.wrap_type[adr+j+1];
      if (type0 == mjhipWRAP_PULLEY || type1 == mjhipWRAP_PULLEY) {
        if (type0 == mjhipWRAP_PULLEY) divisor = m.wrap_prm[adr+j];
        j++;
        continue;
      }
      const bool wrapped = type1 == mjhipWRAP_SPHERE || type1 == mjhipWRAP_CYLINDER;
      const int id0 = m.wrap_objid[adr+j];
      const int id1 = m.wrap_objid[adr + j + (wrapped ? 2 : 1)];
      double wpnt[12], x1[3], wlen = -1;
      int wbody[4];
      for (int k = 0; k < 3; k++) {
        wpnt[k] = d.site_xpos[3*id0 + k];
        x1[k] = d.site_xpos[3*id1 + k];
      }
      wbody[0] = m.site_bodyid[id0];
      int g = -1;
      if (wrapped) {
        g = m.wrap_objid[adr+j+1];
        const int side = (int)lround(m.wrap_prm[adr+j+1]);
        double gpos[3], gmat[9], spos[3];
        for (int k = 0; k < 3; k++) gpos[k] = d.geom_xpos[3*g + k];
        for (int k = 0; k < 9; k++) gmat[k] = d.geom_xmat[9*g + k];
        if (side >= 0) {
          for (int k = 0; k < 3; k++) spos[k] = d.site_xpos[3*side + k];
        }
        wlen = wrapGeom(wpnt + 3, wpnt, x1, gpos, gmat, m.geom_size[3*g], type1,
                        side >= 0 ? spos : nullptr);
      }
      double dif[3];
      if (wlen < 0) {
        copy3(wpnt + 3, x1);
        wbody[1] = m.site_bodyid[id1];
        sub3(dif, wpnt, wpnt + 3);
        d.ten_length[i] += sqrt(dot3(dif, dif)) / divisor;
      } else {
        copy3(wpnt + 9, x1);
        wbody[1] = wbody[2] = m.geom_bodyid[g];
        wbody[3] = m.site_bodyid[id1];
        double d2[3];
        sub3(dif, wpnt, wpnt + 3);
        sub3(d2, wpnt + 6, wpnt + 9);
        d.ten_length[i] += (sqrt(dot3(dif, dif)) + wlen + sqrt(dot3(d2, d2))) / divisor;
      }
      for (int k = 0; k < (wlen < 0 ? 1 : 3); k++) {
        if (wbody[k] == wbody[k+1]) continue;
        sub3(dif, wpnt + 3*k + 3, wpnt + 3*k);
        normalize3(dif);
        SP<S> j1 = d.jact, j2 = d.jact + 3*nv;
        jacInto(m, d, j1, d.jacr, wpnt + 3*k, wbody[k]);
        jacInto(m, d, j2, d.jacr, wpnt + 3*k + 3, wbody[k+1]);
        const double inv = 1/divisor;
        if (sparse) {
          // mj_jacDifPair over the merged chain (its entries are the dense Jacobians' at the
          // chain's dofs), mju_mulMatTVec with dif, then combined into the row
          SP<S, int> chain = d.chainbuf;
          const int NV = mergeChain(m, chain, wbody[k], wbody[k+1]);
          if (!NV) continue;
          for (int p = 0; p < NV; p++) {
            const int c = chain[p];
            double t = 0;
            for (int r = 0; r < 3; r++) {
              if (dif[r]) t += (j2[r*nv + c] - j1[r*nv + c])*dif[r];
            }
            d.jacp[p] = t;
          }
          d.ten_J_rownnz[i] = combineSparse(d.ten_J + radr, d.jacp, 1.0, inv, d.ten_J_rownnz[i],
                                            NV, d.ten_J_colind + radr, chain, d.sparse_buf,
                                            d.chainbuf + 2*nv);
          continue;
        }
        for (int c = 0; c < nv; c++) {   // mju_mulMatTVec of (jac2 - jac1) with dif, then
          double t = 0;                   // mju_addToScl(ten_J row, ., 1/divisor)
          for (int r = 0; r < 3; r++) {
            if (dif[r]) t += (j2[r*nv + c] - j1[r*nv + c])*dif[r];
          }
          d.ten_J[i*nv + c] += t*inv;
        }
      }
      j += wrapped ? 2 : 1;
    }
  }
}

// mj_transmission :865-916 (joint transmission of slide/hinge joints)
template <int S>
MJH_HD void transmission(const mjhipModel& m, const Lane<S>& d, bool after_only = false) {
  for (int i = 0; i < m.nu; i++) {
    int adr = m.moment_rowadr[i];
    int id = m.actuator_trnid[2*i];
    const double* gear = m.actuator_gear + 6*i;
    const int trn = m.actuator_trntype[i];
    if (after_only && !mjh_trnAfter(trn)) continue;
    SP<S> moment = d.actuator_moment + adr;
    if (trn == mjhipTRN_JOINT || trn == mjhipTRN_JOINTINPARENT) {
      const int t = m.jnt_type[id];
      if (t == mjhipJNT_SLIDE || t == mjhipJNT_HINGE) {
        d.actuator_length[i] = d.qpos[m.jnt_qposadr[id]]*gear[0];
        moment[0] = gear[0];
      } else if (t == mjhipJNT_BALL) {     // :912-942 expmap axis . gear axis
        double axis[3], quat[4], gearAxis[3];
        copy4(quat, d.qpos + m.jnt_qposadr[id]);
        normalize4(quat);
        quat2Vel(axis, quat, 1);
        if (trn == mjhipTRN_JOINT) {
          copy3(gearAxis, gear);
        } else {
          quat[1] = -quat[1]; quat[2] = -quat[2]; quat[3] = -quat[3];
          rotVecQuat(gearAxis, gear, quat);
        }
        d.actuator_length[i] = axis[0]*gearAxis[0] + axis[1]*gearAxis[1] + axis[2]*gearAxis[2];
        copy3(moment, gearAxis);
      } else {                              // free joint :944-971
        double gearAxis[3];
        d.actuator_length[i] = 0;
        if (trn == mjhipTRN_JOINT) {
          copy3(gearAxis, gear + 3);
        } else {
          double quat[4];
          copy4(quat, d.qpos + m.jnt_qposadr[id] + 3);
          normalize4(quat);
          quat[1] = -quat[1]; quat[2] = -quat[2]; quat[3] = -quat[3];
          rotVecQuat(gearAxis, gear + 3, quat);
        }
        copy3(moment, gear);
        moment[3] = gearAxis[0]; moment[4] = gearAxis[1]; moment[5] = gearAxis[2];
      }
    } else if (trn == mjhipTRN_SLIDERCRANK) {   // :1000-1052
      const int ids = m.actuator_trnid[2*i+1];
      const double rod = m.actuator_cranklength[i];
      SP<S> smat = d.site_xmat + 9*ids;
      const double axis[3] = {smat[2], smat[5], smat[8]};
      double vec[3], dlda[3], dldv[3];
      sub3(vec, d.site_xpos + 3*id, d.site_xpos + 3*ids);
      const double av = dot3(vec, axis);
      const double det = av*av + rod*rod - dot3(vec, vec);
      if (det <= 0) {                       // crank too short: length = a'v
        d.actuator_length[i] = av;
        copy3(dlda, vec);
        copy3(dldv, axis);
      } else {
        const double sdet = sqrt(det);
        d.actuator_length[i] = av - sdet;
        const double c = 1 - av/sdet, r = 1/sdet;
        for (int k = 0; k < 3; k++) {
          dldv[k] = axis[k]*c;
          dldv[k] += vec[k]*r;
          dlda[k] = vec[k]*c;
        }
      }
      // jacS = d.jacp (slider point), jacA = rotation Jacobian x axis (in d.jacr),
      // jac = crank-site Jacobian - jacS (in d.jacsc)
      const int nv = m.nv;
      jacInto(m, d, d.jacp, d.jacr, d.site_xpos + 3*ids, m.site_bodyid[ids]);
      for (int j = 0; j < nv; j++) {
        const double r0 = d.jacr[j], r1 = d.jacr[nv+j], r2 = d.jacr[2*nv+j];
        d.jacr[j] = r1*axis[2] - r2*axis[1];
        d.jacr[nv+j] = r2*axis[0] - r0*axis[2];
        d.jacr[2*nv+j] = r0*axis[1] - r1*axis[0];
      }
      jacInto(m, d, d.jacsc, d.jacsc + 3*nv, d.site_xpos + 3*id, m.site_bodyid[id]);
      for (int j = 0; j < 3*nv; j++) d.jacsc[j] -= d.jacp[j];
      // dense chain rule into the row (the next rows are written after this one), then
      // gathered to the structural nonzeros (ascending, so in place)
      for (int j = 0; j < nv; j++) {
        double mj = 0;
        for (int k = 0; k < 3; k++) mj += dlda[k]*d.jacr[k*nv+j] + dldv[k]*d.jacsc[k*nv+j];
        moment[j] = mj*gear[0];            // scale by gear ratio (:1039-1043)
      }
      d.actuator_length[i] = d.actuator_length[i]*gear[0];
      for (int k = 0; k < m.moment_rownnz[i]; k++) moment[k] = moment[m.moment_colind[adr+k]];
    } else if (trn == mjhipTRN_SITE) {      // :1084-1225
      const int nv = m.nv;
      double wrench[6];
      jacInto(m, d, d.jacp, d.jacr, d.site_xpos + 3*id, m.site_bodyid[id]);
      d.actuator_length[i] = 0;
      const int refid = m.actuator_trnid[2*i+1];
      if (refid < 0) {                      // gear in the site frame, length 0
        mulMatVec3(wrench, d.site_xmat + 9*id, gear);
        mulMatVec3(wrench + 3, d.site_xmat + 9*id, gear + 3);
        mulMatTVec(moment, d.jacp, wrench, 3, nv);
        mulMatTVec(d.jacp, d.jacr, wrench + 3, 3, nv);
        for (int j = 0; j < nv; j++) moment[j] += d.jacp[j];
      } else {                              // relative to the reference site (:1105-1212)
        // deepest dof shared by the two sites' chains: its chain cancels in the difference
        const int b0 = m.body_weldid[m.site_bodyid[id]], b1 = m.body_weldid[m.site_bodyid[refid]];
        int da0 = m.body_dofadr[b0] + m.body_dofnum[b0] - 1;
        int da1 = m.body_dofadr[b1] + m.body_dofnum[b1] - 1;
        int common = -1;
        if (da0 >= 0 && da1 >= 0) {
          while (da0 != da1) {
            if (da0 < da1) da1 = m.dof_parentid[da1];
            else da0 = m.dof_parentid[da0];
            if (da0 == -1 || da1 == -1) break;
          }
          if (da0 == da1) common = da0;
        }
        for (int j = 0; j < nv; j++) moment[j] = 0;
        SP<S> jref = d.jacsc, jrefr = d.jacsc + 3*nv;
        if (gear[0] != 0 || gear[1] != 0 || gear[2] != 0) {
          double vec[3], loc[3];
          sub3(vec, d.site_xpos + 3*id, d.site_xpos + 3*refid);
          mulMatTVec3(loc, d.site_xmat + 9*refid, vec);
          d.actuator_length[i] += dot3(loc, gear);
          jacInto(m, d, jref, jrefr, d.site_xpos + 3*refid, m.site_bodyid[refid]);
          for (int j = 0; j < 3*nv; j++) d.jacp[j] -= jref[j];
          for (int da = common; da >= 0; da = m.dof_parentid[da]) {
            d.jacp[da] = 0; d.jacp[nv+da] = 0; d.jacp[2*nv+da] = 0;
          }
          mulMatVec3(wrench, d.site_xmat + 9*refid, gear);
          mulMatTVec(moment, d.jacp, wrench, 3, nv);
        }
        if (gear[3] != 0 || gear[4] != 0 || gear[5] != 0) {
          double quat[4], refquat[4], vec[3];
          mulQuat(quat, m.site_quat + 4*id, d.xquat + 4*m.site_bodyid[id]);
          mulQuat(refquat, m.site_quat + 4*refid, d.xquat + 4*m.site_bodyid[refid]);
          subQuat(vec, quat, refquat);
          d.actuator_length[i] += dot3(vec, gear + 3);
          jacInto(m, d, jref, jrefr, d.site_xpos + 3*refid, m.site_bodyid[refid]);
          for (int j = 0; j < 3*nv; j++) d.jacr[j] -= jrefr[j];
          for (int da = common; da >= 0; da = m.dof_parentid[da]) {
            d.jacr[da] = 0; d.jacr[nv+da] = 0; d.jacr[2*nv+da] = 0;
          }
          mulMatVec3(wrench, d.site_xmat + 9*refid, gear + 3);
          mulMatTVec(d.jacp, d.jacr, wrench, 3, nv);
          for (int j = 0; j < nv; j++) moment[j] += d.jacp[j];
        }
      }
      for (int k = 0; k < m.moment_rownnz[i]; k++) moment[k] = moment[m.moment_colind[adr+k]];
    } else if (trn == mjhipTRN_BODY) {      // :1228-1318 adhesion: mean contact normal Jacobian
      const int nv = m.nv, ncon = d.con_count[0];
      d.actuator_length[i] = 0;
      for (int j = 0; j < nv; j++) moment[j] = 0;
      SP<S> mexcl = d.jacsc, jrow = d.jacsc + nv;
      for (int j = 0; j < nv; j++) mexcl[j] = 0;
      int counter = 0;
      // the normal rows' J' * weight in row order (mj_mulJacTVec skips zero weights; the
      // rows of contact j follow those of contact j-1), the in-gap contacts' normal
      // Jacobians on the side
      // sparse mode: mj_mulJacTVec over efc_JT of the weights (d.jar as the reference's
      // efc_force marker array; invConstraint forms jar later)
      const bool sparse = mjh_isSparse(&m);
      if (sparse) {
        for (int r = 0; r < d.efc_count[0]; r++) d.jar[r] = 0;
      }
      for (int c = 0; c < ncon; c++) {
        const int g1 = d.con_geom[2*c], g2 = d.con_geom[2*c+1];
        if (g1 < 0 || g2 < 0) continue;
        const int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
        if (b1 != id && b2 != id) continue;
        const int ex = d.con_exclude[c];
        if (!ex) {
          counter++;
          const int dim = d.con_dim[c], adrc = d.con_efc_address[c];
          const bool one = dim == 1 || m.opt.cone == mjhipCONE_ELLIPTIC;
          const int nr = one ? 1 : 2*(dim - 1);
          const double w = one ? 1.0 : 0.5/(dim - 1);
          for (int r = adrc; r < adrc + nr; r++) {
            if (sparse) {
              d.jar[r] = w;
              continue;
            }
            auto J = d.efc_J + (long)r*nv;
            for (int k = 0; k < nv; k++) moment[k] += J[k]*w;
          }
        } else if (ex == 1) {
          counter++;
          double pos[3], frame[3];
          for (int k = 0; k < 3; k++) { pos[k] = d.con_pos[3*c+k]; frame[k] = d.con_frame[9*c+k]; }
          jacInto(m, d, d.jacp, d.jacr, pos, b1);
          jacInto(m, d, d.jacr, d.jacsc + 2*nv, pos, b2);   // translation only is used
          for (int k = 0; k < nv; k++) jrow[k] = 0;
          for (int q = 0; q < 3; q++) {
            if (frame[q]) {
              for (int k = 0; k < nv; k++) jrow[k] += (d.jacr[q*nv+k] - d.jacp[q*nv+k])*frame[q];
            }
          }
          for (int k = 0; k < nv; k++) mexcl[k] += jrow[k];
        }
      }
      if (counter) {
        if (sparse && d.efc_count[0]) {
          for (int k = 0; k < nv; k++) moment[k] = jacColDot(d, k, d.jar);
        }
        const double s = -1.0/counter;
        for (int k = 0; k < nv; k++) {
          moment[k] += mexcl[k];
          moment[k] = moment[k]*s;
        }
      }
      for (int k = 0; k < m.moment_rownnz[i]; k++) moment[k] = moment[m.moment_colind[adr+k]];
    } else if (mjh_isSparse(&m)) {          // tendon, sparse (:1060-1067): the tendon's row
      d.actuator_length[i] = d.ten_length[id]*gear[0];
      const int tadr = d.ten_J_rowadr[id];
      for (int k = 0; k < m.moment_rownnz[i]; k++) moment[k] = d.ten_J[tadr + k]*gear[0];
    } else {                                // fixed tendon :1053-1081 (model-constant nonzeros)
      d.actuator_length[i] = d.ten_length[id]*gear[0];
      for (int k = 0; k < m.moment_rownnz[i]; k++) {
        moment[k] = d.ten_J[id*m.nv + m.moment_colind[adr+k]]*gear[0];
      }
    }
  }
}

// mj_crb :1353-1401
template <int S>
MJH_HD void crb(const mjhipModel& m, const Lane<S>& d) {
  double buf[6];
  int nv = m.nv;
  copy(d.crb, d.cinert, 10*m.nbody);
  for (int i = m.nbody - 1; i > 0; i--) {
    if (m.body_parentid[i] > 0) addTo(d.crb + 10*m.body_parentid[i], d.crb + 10*i, 10);
  }
  zero(d.qM, m.nM);
  for (int i = 0; i < nv; i++) {
    if (m.dof_simplenum[i]) {
      int n = i + m.dof_simplenum[i];
      for (; i < n; i++) d.qM[m.dof_Madr[i]] = m.dof_M0[i];
      if (i == nv) break;
    }
    int Madr_ij = m.dof_Madr[i];
    d.qM[Madr_ij] = m.dof_armature[i];
    mulInertVec(buf, d.crb + 10*m.dof_bodyid[i], d.cdof + 6*i);
    for (int j = i; j >= 0; j = m.dof_parentid[j]) {
      d.qM[Madr_ij++] += dot6(d.cdof + 6*j, buf);
    }
  }
}

// mj_factorM / mj_factorI :1470-1511. A pivot below mjMINVAL (or NaN) sets
// MJHIP_INST_INERTIA, the condition mj_factorI_legacy reports as mjWARN_INERTIA (:1426-1430);
// the factor itself is left as mj_factorI computes it (no clamping on this path)
template <int S>
MJH_HD void factorM(const mjhipModel& m, const Lane<S>& d, int* status = nullptr) {
  for (int i = 0; i < m.nC; i++) d.qLD[i] = d.qM[m.mapM2C[i]];
  SP<S> mat = d.qLD;
  const int *rownnz = m.C_rownnz, *rowadr = m.C_rowadr, *colind = m.C_colind;
  for (int k = m.nv-1; k >= 0; k--) {
    int rowadr_k = rowadr[k];
    int diag_k = rowadr_k + rownnz[k] - 1;
    if (status && !(mat[diag_k] >= MINVAL)) *status |= MJHIP_INST_INERTIA;
    double invD = 1 / mat[diag_k];
    d.qLDiagInv[k] = invD;
    if (m.dof_simplenum[k]) continue;
    for (int adr = diag_k - 1; adr >= rowadr_k; adr--) {
      double tmp = mat[adr] * invD;
      int i = colind[adr];
      addToScl(mat + rowadr[i], mat + rowadr_k, -tmp, rownnz[i]);
      mat[adr] = tmp;
    }
  }
}

// mj_comVel :1833-1896
template <int S>
MJH_HD void comVel(const mjhipModel& m, const Lane<S>& d) {
  zero(d.cvel, 6);
  for (int i = 1; i < m.nbody; i++) {
    int bda = m.body_dofadr[i];
    double cvel[6];
    copy(cvel, d.cvel + 6*m.body_parentid[i], 6);
    int dofnum = m.body_dofnum[i];
    for (int j = 0; j < dofnum; j++) {
      double tmp[6];
      switch (m.jnt_type[m.dof_jntid[bda + j]]) {
      case mjhipJNT_FREE:
        zero(d.cdof_dot + 6*bda, 18);
        mulDofVec(tmp, d.cdof + 6*bda, d.qvel + bda, 3);
        addTo(cvel, tmp, 6);
        j += 3;
        // fallthrough
      case mjhipJNT_BALL:
        for (int k = 0; k < 3; k++) {
          crossMotion(d.cdof_dot + 6*(bda + j + k), cvel, d.cdof + 6*(bda + j + k));
        }
        mulDofVec(tmp, d.cdof + 6*(bda + j), d.qvel + bda + j, 3);
        addTo(cvel, tmp, 6);
        j += 2;
        break;
      default:
        crossMotion(d.cdof_dot + 6*(bda + j), cvel, d.cdof + 6*(bda + j));
        mulDofVec(tmp, d.cdof + 6*(bda + j), d.qvel + bda + j, 1);
        addTo(cvel, tmp, 6);
      }
    }
    copy(d.cvel + 6*i, cvel, 6);
  }
}

// mj_rne :1969-2023 (result = null: only the mirror's scratch)
template <int S>
MJH_HD void rne(const mjhipModel& m, const Lane<S>& d, int flg_acc, SP<S> result) {
  int nbody = m.nbody, nv = m.nv;
  double tmp[6], tmp1[6];
  SP<S> cacc = d.cacc, cfrc = d.cfrc;
  zero(cacc, 6);
  if (!(m.opt.disableflags & mjhipDSBL_GRAVITY)) scl3(cacc + 3, m.opt.gravity, -1);
  for (int i = 1; i < nbody; i++) {
    int bda = m.body_dofadr[i];
    mulDofVec(tmp, d.cdof_dot + 6*bda, d.qvel + bda, m.body_dofnum[i]);
    add(cacc + 6*i, cacc + 6*m.body_parentid[i], tmp, 6);
    if (flg_acc) {
      mulDofVec(tmp, d.cdof + 6*bda, d.qacc + bda, m.body_dofnum[i]);
      addTo(cacc + 6*i, tmp, 6);
    }
    mulInertVec(cfrc + 6*i, d.cinert + 10*i, cacc + 6*i);
    mulInertVec(tmp, d.cinert + 10*i, d.cvel + 6*i);
    crossForce(tmp1, d.cvel + 6*i, tmp);
    addTo(cfrc + 6*i, tmp1, 6);
  }
  zero(cfrc, 6);
  for (int i = nbody - 1; i > 0; i--) {
    if (m.body_parentid[i]) addTo(cfrc + 6*m.body_parentid[i], cfrc + 6*i, 6);
  }
  for (int i = 0; i < nv; i++) {
    result[i] = dot6(d.cdof + 6*i, cfrc + 6*m.dof_bodyid[i]);
  }
}

//---------------------------------- engine_passive.c -----------------------------------------

// mj_passive :436-493 with mj_springdamper :57-378 and mj_gravcomp :381-399
template <int S, class R>
MJH_HD void objectVelocity(const mjhipModel& m, const Lane<S>& d, int type, int id, R res,
                           int flg_local);
template <class R, class V, class P, class O, class M>
MJH_HD void transformSpatial(R res, V vec, int flg_force, P newpos, O oldpos, M rot,
                             bool has_rot);

// engine_passive.c:527-585 mj_inertiaBoxFluidModel: viscous and quadratic drag of the body's
// equivalent inertia box, at the COM
template <int S>
MJH_HD void inertiaBoxFluid(const mjhipModel& m, const Lane<S>& d, int i) {
  double lvel[6], wind[6], lwind[6], lfrc[6], bfrc[6], box[3];
  const double* inertia = m.body_inertia + 3*i;
  const double mass = m.body_mass[i];
  auto mx = [](double a, double b) { return a > b ? a : b; };   // mju_max
  box[0] = sqrt(mx(MINVAL, (inertia[1] + inertia[2] - inertia[0])) / mass * 6.0);
  box[1] = sqrt(mx(MINVAL, (inertia[0] + inertia[2] - inertia[1])) / mass * 6.0);
  box[2] = sqrt(mx(MINVAL, (inertia[0] + inertia[1] - inertia[2])) / mass * 6.0);
  objectVelocity(m, d, 1, i, lvel, 1);
  for (int k = 0; k < 3; k++) { wind[k] = 0; wind[3 + k] = m.opt.wind[k]; }
  transformSpatial(lwind, wind, 0, d.xipos + 3*i, d.subtree_com + 3*m.body_rootid[i],
                   d.ximat + 9*i, true);
  lvel[3] -= lwind[3]; lvel[4] -= lwind[4]; lvel[5] -= lwind[5];
  for (int k = 0; k < 6; k++) lfrc[k] = 0;
  const double visc = m.opt.viscosity, dens = m.opt.density;
  if (visc > 0) {
    const double diam = (box[0] + box[1] + box[2])/3.0;
    scl3(lfrc, lvel, -mjhipPI*diam*diam*diam*visc);
    scl3(lfrc + 3, lvel + 3, -3.0*mjhipPI*diam*visc);
  }
  if (dens > 0) {
    lfrc[3] -= 0.5*dens*box[1]*box[2]*fabs(lvel[3])*lvel[3];
    lfrc[4] -= 0.5*dens*box[0]*box[2]*fabs(lvel[4])*lvel[4];
    lfrc[5] -= 0.5*dens*box[0]*box[1]*fabs(lvel[5])*lvel[5];
    lfrc[0] -= dens*box[0]*(box[1]*box[1]*box[1]*box[1]+box[2]*box[2]*box[2]*box[2])*
               fabs(lvel[0])*lvel[0]/64.0;
    lfrc[1] -= dens*box[1]*(box[0]*box[0]*box[0]*box[0]+box[2]*box[2]*box[2]*box[2])*
               fabs(lvel[1])*lvel[1]/64.0;
    lfrc[2] -= dens*box[2]*(box[0]*box[0]*box[0]*box[0]+box[1]*box[1]*box[1]*box[1])*
               fabs(lvel[2])*lvel[2]/64.0;
  }
  mulMatVec3(bfrc, d.ximat + 9*i, lfrc);
  mulMatVec3(bfrc + 3, d.ximat + 9*i, lfrc + 3);
  applyFT(m, d, bfrc + 3, bfrc, d.xipos + 3*i, i, d.qfrc_fluid);
}

// engine_passive.c:650-687 mj_addedMassForces (no accelerations: the reference passes none)
MJH_HD void addedMassForces(const double v[6], double rho, const double* vm, const double* vi,
                            double f[6]) {
  const double lin[3] = {v[3], v[4], v[5]}, ang[3] = {v[0], v[1], v[2]};
  const double plin[3] = {rho*vm[0]*lin[0], rho*vm[1]*lin[1], rho*vm[2]*lin[2]};
  const double pang[3] = {rho*vi[0]*ang[0], rho*vi[1]*ang[1], rho*vi[2]*ang[2]};
  double fa[3], t1[3], t2[3];
  cross(fa, plin, ang);
  cross(t1, plin, lin);
  cross(t2, pang, ang);
  addTo3(f, t1);
  addTo3(f, t2);
  addTo3(f + 3, fa);
}

MJH_HD double pow4(double x) { return (x*x)*(x*x); }

// engine_passive.c:705-790 mj_viscousForces: Magnus and Kutta-Joukowski lift, Stokes and
// quadratic (blunt/slender) drag of the equivalent ellipsoid with semi-axes s
MJH_HD void viscousForces(const double v[6], double rho, double mu, const double s[3],
                          double magnus, double kutta, double blunt, double slender,
                          double angdrag, double f[6]) {
  auto mx = [](double a, double b) { return a > b ? a : b; };
  auto mn = [](double a, double b) { return a < b ? a : b; };
  const double lin[3] = {v[3], v[4], v[5]}, ang[3] = {v[0], v[1], v[2]};
  const double volume = 4.0/3.0 * mjhipPI * s[0] * s[1] * s[2];
  const double dmax = mx(mx(s[0], s[1]), s[2]);
  const double dmin = mn(mn(s[0], s[1]), s[2]);
  const double dmid = s[0] + s[1] + s[2] - dmax - dmin;
  const double Amax = mjhipPI * dmax * dmid;
  double mf[3];
  cross(mf, ang, lin);
  mf[0] *= magnus * rho * volume;
  mf[1] *= magnus * rho * volume;
  mf[2] *= magnus * rho * volume;
  const double den = pow4(s[1]*s[2]) * (lin[0]*lin[0]) + pow4(s[2]*s[0]) * (lin[1]*lin[1]) +
                     pow4(s[0]*s[1]) * (lin[2]*lin[2]);
  const double num = (s[1]*s[2]*lin[0])*(s[1]*s[2]*lin[0]) +
                     (s[2]*s[0]*lin[1])*(s[2]*s[0]*lin[1]) +
                     (s[0]*s[1]*lin[2])*(s[0]*s[1]*lin[2]);
  const double Aproj = mjhipPI * sqrt(den/mx(MINVAL, num));
  const double nrm[3] = {(s[1]*s[2])*(s[1]*s[2]) * lin[0], (s[2]*s[0])*(s[2]*s[0]) * lin[1],
                         (s[0]*s[1])*(s[0]*s[1]) * lin[2]};
  const double linn = sqrt(lin[0]*lin[0] + lin[1]*lin[1] + lin[2]*lin[2]);
  const double cosa = num / mx(MINVAL, linn * den);
  double kc[3], kf[3];
  cross(kc, nrm, lin);
  kc[0] *= kutta * rho * cosa * Aproj;
  kc[1] *= kutta * rho * cosa * Aproj;
  kc[2] *= kutta * rho * cosa * Aproj;
  cross(kf, kc, lin);
  const double D = 2.0/3.0 * (s[0] + s[1] + s[2]);
  const double cf = 3.0 * mjhipPI * D, ct = mjhipPI * D*D*D;
  const double Imax = 8.0/15.0 * mjhipPI * dmid * pow4(dmax);
  double II[3];
  for (int k = 0; k < 3; k++) {          // mji_ellipsoid_max_moment (:697-701)
    II[k] = 8.0/15.0 * mjhipPI * s[k] * pow4(mx(s[(k+1) % 3], s[(k+2) % 3]));
  }
  const double mom[3] = {ang[0] * (angdrag*II[0] + slender*(Imax - II[0])),
                         ang[1] * (angdrag*II[1] + slender*(Imax - II[1])),
                         ang[2] * (angdrag*II[2] + slender*(Imax - II[2]))};
  const double dlin = mu*cf + rho*linn*(Aproj*blunt + slender*(Amax - Aproj));
  const double dang = mu * ct + rho * sqrt(mom[0]*mom[0] + mom[1]*mom[1] + mom[2]*mom[2]);
  f[0] -= dang * ang[0];
  f[1] -= dang * ang[1];
  f[2] -= dang * ang[2];
  f[3] += mf[0] + kf[0] - dlin*lin[0];
  f[4] += mf[1] + kf[1] - dlin*lin[1];
  f[5] += mf[2] + kf[2] - dlin*lin[2];
}

// engine_passive.c:588-646 mj_ellipsoidFluidModel over body b's geoms (geom_fluid holds the
// compiler's coefficients: readFluidGeomInteraction :793-821)
template <int S>
MJH_HD void ellipsoidFluid(const mjhipModel& m, const Lane<S>& d, int b) {
  for (int j = 0; j < m.body_geomnum[b]; j++) {
    const int g = m.body_geomadr[b] + j;
    const double* c = m.geom_fluid + 12*g;
    const double* sz = m.geom_size + 3*g;
    double ax[3];                         // mju_geomSemiAxes (engine_util_misc.c:425-451)
    const int t = m.geom_type[g];
    if (t == mjhipGEOM_SPHERE) { ax[0] = sz[0]; ax[1] = sz[0]; ax[2] = sz[0]; }
    else if (t == mjhipGEOM_CAPSULE) { ax[0] = sz[0]; ax[1] = sz[0]; ax[2] = sz[1] + sz[0]; }
    else if (t == mjhipGEOM_CYLINDER) { ax[0] = sz[0]; ax[1] = sz[0]; ax[2] = sz[1]; }
    else { ax[0] = sz[0]; ax[1] = sz[1]; ax[2] = sz[2]; }
    if (c[0] == 0.0) continue;
    double lvel[6], wind[6], lwind[6], lfrc[6], bfrc[6];
    objectVelocity(m, d, 5, g, lvel, 1);  // mjOBJ_GEOM
    for (int k = 0; k < 3; k++) { wind[k] = 0; wind[3 + k] = m.opt.wind[k]; }
    transformSpatial(lwind, wind, 0, d.geom_xpos + 3*g, d.subtree_com + 3*m.body_rootid[b],
                     d.geom_xmat + 9*g, true);
    lvel[3] -= lwind[3]; lvel[4] -= lwind[4]; lvel[5] -= lwind[5];
    for (int k = 0; k < 6; k++) lfrc[k] = 0;
    addedMassForces(lvel, m.opt.density, c + 6, c + 9, lfrc);
    viscousForces(lvel, m.opt.density, m.opt.viscosity, ax, c[5], c[4], c[1], c[2], c[3], lfrc);
    for (int k = 0; k < 6; k++) lfrc[k] = lfrc[k]*c[0];
    mulMatVec3(bfrc, d.geom_xmat + 9*g, lfrc);
    mulMatVec3(bfrc + 3, d.geom_xmat + 9*g, lfrc + 3);
    applyFT(m, d, bfrc + 3, bfrc, d.geom_xpos + 3*g, b, d.qfrc_fluid);
  }
}

template <int S>
MJH_HD void passive(const mjhipModel& m, const Lane<S>& d) {
  int nv = m.nv;
  zero(d.qfrc_spring, nv);
  zero(d.qfrc_damper, nv);
  zero(d.qfrc_gravcomp, nv);
  zero(d.qfrc_fluid, nv);
  zero(d.qfrc_passive, nv);
  if (m.opt.disableflags & mjhipDSBL_PASSIVE) return;
  for (int i = 0; i < m.njnt; i++) {
    double stiffness = m.jnt_stiffness[i];
    if (stiffness == 0) continue;
    int padr = m.jnt_qposadr[i];
    int dadr = m.jnt_dofadr[i];
    switch (m.jnt_type[i]) {
    case mjhipJNT_FREE:
      d.qfrc_spring[dadr+0] = -stiffness*(d.qpos[padr+0] - m.qpos_spring[padr+0]);
      d.qfrc_spring[dadr+1] = -stiffness*(d.qpos[padr+1] - m.qpos_spring[padr+1]);
      d.qfrc_spring[dadr+2] = -stiffness*(d.qpos[padr+2] - m.qpos_spring[padr+2]);
      dadr += 3;
      padr += 3;
      // fallthrough
    case mjhipJNT_BALL:
      {
        double dif[3], quat[4];
        copy4(quat, d.qpos + padr);
        normalize4(quat);
        subQuat(dif, quat, m.qpos_spring + padr);
        d.qfrc_spring[dadr+0] = -stiffness*dif[0];
        d.qfrc_spring[dadr+1] = -stiffness*dif[1];
        d.qfrc_spring[dadr+2] = -stiffness*dif[2];
      }
      break;
    default:
      d.qfrc_spring[dadr] = -stiffness*(d.qpos[padr] - m.qpos_spring[padr]);
      break;
    }
  }
  for (int i = 0; i < nv; i++) {
    double damping = m.dof_damping[i];
    if (damping != 0) d.qfrc_damper[i] = -damping*d.qvel[i];
  }
  for (int i = 0; i < m.ntendon; i++) {
    double stiffness = m.tendon_stiffness[i];
    double damping = m.tendon_damping[i];
    if (stiffness == 0 && damping == 0) continue;
    double length = d.ten_length[i];
    double lower = m.tendon_lengthspring[2*i];
    double upper = m.tendon_lengthspring[2*i+1];
    double frc_spring = 0;
    if (length > upper) {
      frc_spring = stiffness * (upper - length);
    } else if (length < lower) {
      frc_spring = stiffness * (lower - length);
    }
    double frc_damper = -damping * d.ten_velocity[i];
    if (mjh_isSparse(&m)) {                // :361-370 over the tendon's compressed row
      if (frc_spring || frc_damper) {
        const int a = d.ten_J_rowadr[i], e = a + d.ten_J_rownnz[i];
        for (int j = a; j < e; j++) {
          const int k = d.ten_J_colind[j];
          const double J = d.ten_J[j];
          d.qfrc_spring[k] += J * frc_spring;
          d.qfrc_damper[k] += J * frc_damper;
        }
      }
      continue;
    }
    if (frc_spring) addToScl(d.qfrc_spring, d.ten_J + i*nv, frc_spring, nv);
    if (frc_damper) addToScl(d.qfrc_damper, d.ten_J + i*nv, frc_damper, nv);
  }
  int has_gravcomp = 0;
  const double* g = m.opt.gravity;
  if (m.ngravcomp && !(m.opt.disableflags & mjhipDSBL_GRAVITY) &&
      sqrt(g[0]*g[0] + g[1]*g[1] + g[2]*g[2]) != 0) {
    for (int i = 1; i < m.nbody; i++) {
      if (m.body_gravcomp[i]) {
        has_gravcomp = 1;
        double force[3];
        scl3(force, g, -(m.body_mass[i]*m.body_gravcomp[i]));
        applyForce(m, d, force, d.xipos + 3*i, i, d.qfrc_gravcomp);
      }
    }
  }
  // fluid forces (mj_fluid engine_passive.c:402-428): the ellipsoid model for a body with a
  // geom that uses it, the inertia-box model otherwise
  const bool has_fluid = m.opt.viscosity > 0 || m.opt.density > 0;
  if (has_fluid) {
    for (int i = 1; i < m.nbody; i++) {
      if (m.body_mass[i] < MINVAL) continue;
      int ell = 0;
      for (int j = 0; j < m.body_geomnum[i] && ell == 0; j++) {
        ell += m.geom_fluid[12*(m.body_geomadr[i] + j)] > 0;
      }
      if (ell) ellipsoidFluid(m, d, i);
      else inertiaBoxFluid(m, d, i);
    }
  }
  add(d.qfrc_passive, d.qfrc_spring, d.qfrc_damper, nv);
  if (has_fluid) addTo(d.qfrc_passive, d.qfrc_fluid, nv);
  if (has_gravcomp) {
    for (int i = 0; i < m.njnt; i++) {
      if (m.jnt_actgravcomp[i]) continue;
      int t = m.jnt_type[i];
      int dofnum = t == mjhipJNT_FREE ? 6 : (t == mjhipJNT_BALL ? 3 : 1);
      int dofadr = m.jnt_dofadr[i];
      for (int j = 0; j < dofnum; j++) d.qfrc_passive[dofadr+j] += d.qfrc_gravcomp[dofadr+j];
    }
  }
}

//---------------------------------- engine_core_constraint.c ---------------------------------

// row counters of mj_makeConstraint (nefc, equality, friction and limit rows), kept in
// registers and written to efc_count once at the end
struct RowCount { int nefc = 0, ne = 0, nf = 0, nl = 0; };

//------------------- compressed rows of sparse-mode models (mjh_isSparse) --------------------

// mj_mergeChain engine_support.c:264-304 / mj_mergeChainSimple :309-336: the merged dof chain
// of two bodies, increasing, into chain; returns its length
template <class C>
MJH_HD int mergeChain(const mjhipModel& m, C chain, int b1, int b2) {
  if (m.body_simple[b1] && m.body_simple[b2]) {
    if (b1 > b2) { const int t = b1; b1 = b2; b2 = t; }
    const int n1 = m.body_dofnum[b1], n2 = m.body_dofnum[b2];
    for (int i = 0; i < n1; i++) chain[i] = m.body_dofadr[b1] + i;
    for (int i = 0; i < n2; i++) chain[n1+i] = m.body_dofadr[b2] + i;
    return n1 + n2;
  }
  while (b1 && !m.body_dofnum[b1]) b1 = m.body_parentid[b1];
  while (b2 && !m.body_dofnum[b2]) b2 = m.body_parentid[b2];
  if (b1 == 0 && b2 == 0) return 0;
  int da1 = m.body_dofadr[b1] + m.body_dofnum[b1] - 1;
  int da2 = m.body_dofadr[b2] + m.body_dofnum[b2] - 1;
  int NV = 0;
  while (da1 >= 0 || da2 >= 0) {
    const int c = da1 > da2 ? da1 : da2;
    chain[NV++] = c;
    if (da1 == c) da1 = m.dof_parentid[da1];
    if (da2 == c) da2 = m.dof_parentid[da2];
  }
  for (int i = 0; i < NV/2; i++) {
    const int t = chain[i];
    chain[i] = chain[NV-i-1];
    chain[NV-i-1] = t;
  }
  return NV;
}

// mju_combineSparse engine_util_sparse.h:244-303: dst = a*dst + b*src over the union of the two
// index sets (buf, buf_ind: scratch of nv entries); returns the result's nnz
template <class D, class DI, class V, class VI, class B, class BI>
MJH_HD int combineSparse(D dst, V src, double a, double b, int dst_nnz, int src_nnz, DI dst_ind,
                         VI src_ind, B buf, BI buf_ind) {
  bool same = dst_nnz == src_nnz;
  for (int i = 0; same && i < dst_nnz; i++) same = dst_ind[i] == src_ind[i];
  if (same) {
    for (int i = 0; i < dst_nnz; i++) dst[i] = dst[i]*a + src[i]*b;   // mju_addToSclScl
    return dst_nnz;
  }
  for (int i = 0; i < dst_nnz; i++) {
    buf[i] = dst[i];
    buf_ind[i] = dst_ind[i];
  }
  int bi = 0, si = 0, nnz = 0;
  while (bi < dst_nnz && si < src_nnz) {
    const int badr = buf_ind[bi], sadr = src_ind[si];
    if (badr == sadr) {
      dst[nnz] = a*buf[bi++] + b*src[si++];
      dst_ind[nnz++] = badr;
    } else if (badr < sadr) {
      dst[nnz] = a*buf[bi++];
      dst_ind[nnz++] = badr;
    } else {
      dst[nnz] = b*src[si++];
      dst_ind[nnz++] = sadr;
    }
  }
  while (si < src_nnz) {
    dst[nnz] = b*src[si];
    dst_ind[nnz++] = src_ind[si++];
  }
  while (bi < dst_nnz) {
    dst[nnz] = a*buf[bi];
    dst_ind[nnz++] = buf_ind[bi++];
  }
  return nnz;
}

// mj_addConstraint :300-331, sparse branch: `size` rows of NV values each (jac, row-major
// size x NV) over `chain`, appended to the compressed rows; returns false when the rows were
// not added (an empty chain of a non-contact row, or the capacity)
template <int S, class J, class C>
MJH_HD bool addRowsSparse(const mjhipModel& m, const Lane<S>& d, RowCount& rc, J jac, int NV,
                          C chain, const double* pos, const double* margin, double frictionloss,
                          int size, int type, int id, int* status) {
  const bool contact = type == CNSTR_CONTACT_FRICTIONLESS || type == CNSTR_CONTACT_PYRAMIDAL ||
                       type == CNSTR_CONTACT_ELLIPTIC;
  NV = NV > 0 ? NV : 0;
  if (!NV && !contact) return false;
  const int nefc = rc.nefc;
  const int adr0 = nefc ? d.efc_J_rowadr[nefc-1] + d.efc_J_rownnz[nefc-1] : 0;
  if (nefc + size > d.efc_cap || adr0 + (long)size*NV > d.nj_cap) {
    *status |= MJHIP_INST_CNSTRFULL;   // mjWARN_CNSTRFULL analogue: capacity exceeded
    return false;
  }
  for (int i = 0; i < size; i++) {
    const int adr = adr0 + i*NV;
    d.efc_J_rowadr[nefc+i] = adr;
    d.efc_J_rownnz[nefc+i] = NV;
    for (int k = 0; k < NV; k++) {
      d.efc_J_colind[adr+k] = chain[k];
      d.efc_J[adr+k] = jac[i*NV+k];
    }
  }
  for (int i = 0; i < size; i++) {
    d.efc_pos[nefc+i] = pos ? pos[i] : 0;
    d.efc_margin[nefc+i] = margin ? margin[i] : 0;
    d.efc_frictionloss[nefc+i] = frictionloss;
    d.efc_type[nefc+i] = type;
    d.efc_id[nefc+i] = id;
  }
  rc.nefc = nefc + size;
  if (type == CNSTR_EQUALITY) {
    rc.ne += size;
  } else if (type == CNSTR_FRICTION_DOF || type == CNSTR_FRICTION_TENDON) {
    rc.nf += size;
  } else if (type == CNSTR_LIMIT_JOINT || type == CNSTR_LIMIT_TENDON) {
    rc.nl += size;
  }
  return true;
}

// mju_transposeSparse engine_util_sparse.c:474-515: efc_JT from the compressed efc_J rows.
// The rows of one contact share its chain (instantiateContact), so they are transposed as a
// group: one count and one slot update per chain column for the whole group, its rows then
// written to consecutive slots in row order -- the same efc_JT, with a quarter of the
// read-modify-write round trips on the per-column counters (each waits for the previous one
// in memory) for pyramidal contacts.
template <int S>
MJH_HD int transposeGroup(const Lane<S>& d, int r, int nefc) {
  const int t = d.efc_type[r];
  if (t != CNSTR_CONTACT_FRICTIONLESS && t != CNSTR_CONTACT_PYRAMIDAL &&
      t != CNSTR_CONTACT_ELLIPTIC) {
    return 1;
  }
  const int id = d.efc_id[r];
  int g = 1;
  while (r + g < nefc && d.efc_id[r + g] == id && d.efc_type[r + g] == t) g++;
  return g;
}

template <int S>
MJH_HD void transposeRows(const mjhipModel& m, const Lane<S>& d, int nefc) {
  const int nv = m.nv;
  for (int j = 0; j < nv; j++) d.efc_JT_rownnz[j] = 0;
  for (int r = 0; r < nefc;) {
    const int g = transposeGroup(d, r, nefc);
    const int a = d.efc_J_rowadr[r], e = a + d.efc_J_rownnz[r];
    for (int k = a; k < e; k++) {
      const int c = d.efc_J_colind[k];
      d.efc_JT_rownnz[c] = d.efc_JT_rownnz[c] + g;
    }
    r += g;
  }
  int acc = 0;
  for (int j = 0; j < nv; j++) {             // rowadr as the next free slot of each row
    d.efc_JT_rowadr[j] = acc;
    acc += d.efc_JT_rownnz[j];
  }
  for (int r = 0; r < nefc;) {
    const int g = transposeGroup(d, r, nefc);
    const int a = d.efc_J_rowadr[r], n = d.efc_J_rownnz[r];
    for (int k = 0; k < n; k++) {
      const int c = d.efc_J_colind[a + k];
      const int slot = d.efc_JT_rowadr[c];
      d.efc_JT_rowadr[c] = slot + g;
      for (int i = 0; i < g; i++) {            // row r+i's entry k (rows of a group: stride n)
        d.efc_JT_colind[slot + i] = r + i;
        d.efc_JT[slot + i] = d.efc_J[a + i*n + k];
      }
    }
    r += g;
  }
  for (int j = 0; j < nv; j++) d.efc_JT_rowadr[j] = d.efc_JT_rowadr[j] - d.efc_JT_rownnz[j];
}

// mj_mulJacVec :361-377 / mj_mulJacTVec :426-442 of a sparse-mode model: mju_mulMatVecSparse
// over the rows of efc_J / efc_JT
template <int S, class V>
MJH_HD double jacRowDot(const Lane<S>& d, int r, V vec) {
  const int a = d.efc_J_rowadr[r];
  return dotSparse(d.efc_J + a, vec, d.efc_J_rownnz[r], d.efc_J_colind + a);
}
template <int S, class V>
MJH_HD double jacColDot(const Lane<S>& d, int j, V vec) {
  const int a = d.efc_JT_rowadr[j];
  return dotSparse(d.efc_JT + a, vec, d.efc_JT_rownnz[j], d.efc_JT_colind + a);
}

// mj_addConstraint :265-356 (dense): `size` rows of jac (strided scratch), contact rows are
// never dropped as empty. Returns whether the rows were added. Sparse-mode models come with
// their row's chain (jac is then size x NV) and take the compressed branch.
template <int S>
MJH_HD bool addConstraint(const mjhipModel& m, const Lane<S>& d, RowCount& rc, SP<S> jac,
                          const double* pos, const double* margin, double frictionloss,
                          int size, int type, int id, int* status, int NV = 0,
                          SP<S, int> chain = SP<S, int>{nullptr}) {
  if (mjh_isSparse(&m)) {
    return addRowsSparse(m, d, rc, jac, NV, chain, pos, margin, frictionloss, size, type, id,
                         status);
  }
  int nv = m.nv;
  int nefc = rc.nefc;
  int empty = !(type == CNSTR_CONTACT_FRICTIONLESS || type == CNSTR_CONTACT_PYRAMIDAL ||
                type == CNSTR_CONTACT_ELLIPTIC);
  for (int i = 0; empty && i < size*nv; i++) {
    if (jac[i]) empty = 0;
  }
  if (empty) return false;
  if (nefc + size > d.efc_cap) {   // mjWARN_CNSTRFULL analogue: capacity exceeded
    *status |= MJHIP_INST_CNSTRFULL;
    return false;
  }
  copy(d.efc_J + nefc*nv, jac, size*nv);
  for (int i = 0; i < size; i++) {
    d.efc_pos[nefc+i] = pos ? pos[i] : 0;
    d.efc_margin[nefc+i] = margin ? margin[i] : 0;
    d.efc_frictionloss[nefc+i] = frictionloss;
    d.efc_type[nefc+i] = type;
    d.efc_id[nefc+i] = id;
  }
  rc.nefc = nefc + size;
  if (type == CNSTR_EQUALITY) {
    rc.ne += size;
  } else if (type == CNSTR_FRICTION_DOF || type == CNSTR_FRICTION_TENDON) {
    rc.nf += size;
  } else if (type == CNSTR_LIMIT_JOINT || type == CNSTR_LIMIT_TENDON) {
    rc.nl += size;
  }
  return true;
}

template <int S>
MJH_HD bool addConstraint1(const mjhipModel& m, const Lane<S>& d, RowCount& rc, SP<S> jacrow,
                           double pos, double margin, double frictionloss, int type, int id,
                           int* status, int NV = 0, SP<S, int> chain = SP<S, int>{nullptr}) {
  return addConstraint(m, d, rc, jacrow, &pos, &margin, frictionloss, 1, type, id, status, NV,
                       chain);
}

// mj_instantiateContact :964-1131 (dense; pyramidal or frictionless; elliptic cones are
// rejected with contacts at context creation). The reference forms the two body Jacobians
// (mj_jacDifPair), their difference, its rotation into the contact frame (mju_mulMatMat)
// and the pyramid rows as dense nv-arrays. Every element of those depends only on its own
// dof, so the rows are formed here dof by dof, in the same order of operations (including
// mju_mulMatMat's skip of zero frame entries), straight into efc_J: no Jacobian scratch.
MJH_HD bool ancestorOrSelf(const mjhipModel& m, int a, int b) {
  while (b > a) b = m.body_parentid[b];   // body ids are depth-first: parents come first
  return b == a;
}

template <int S>
MJH_HD void instantiateContact(const mjhipModel& m, const Lane<S>& d, RowCount& rc,
                               int* status) {
  int nv = m.nv, ncon = d.con_count[0];
  if ((m.opt.disableflags & mjhipDSBL_CONTACT) || ncon == 0 || nv == 0) return;
  const bool elliptic = m.opt.cone == mjhipCONE_ELLIPTIC;
  for (int i = 0; i < ncon; i++) {
    if (d.con_exclude[i]) continue;
    const int dim = d.con_dim[i];
    const int rows = mjhip_contactRows(dim, elliptic);
    const int nefc = rc.nefc;
    d.con_efc_address[i] = nefc;
    if (nefc + rows > d.efc_cap) {   // mjWARN_CNSTRFULL analogue (capacity is exact)
      *status |= MJHIP_INST_CNSTRFULL;
      continue;
    }
    const int b1 = m.geom_bodyid[d.con_geom[2*i]], b2 = m.geom_bodyid[d.con_geom[2*i+1]];
    // dense rows of nv values, or (sparse mode) compressed rows over the bodies' merged chain
    // (mj_jacDifPair :659-731; a contact whose chain is empty is excluded, :1071-1076)
    const bool sparse = mjh_isSparse(&m);
    SP<S, int> chain = d.chainbuf;
    int NV = nv;
    long adr0 = (long)nefc*nv;
    if (sparse) {
      NV = mergeChain(m, chain, b1, b2);
      if (!NV) {
        d.con_efc_address[i] = -1;
        d.con_exclude[i] = 3;
        continue;
      }
      adr0 = nefc ? d.efc_J_rowadr[nefc-1] + d.efc_J_rownnz[nefc-1] : 0;
      if (adr0 + (long)rows*NV > d.nj_cap) {
        *status |= MJHIP_INST_CNSTRFULL;
        continue;
      }
      for (int r = 0; r < rows; r++) {
        d.efc_J_rowadr[nefc + r] = (int)(adr0 + (long)r*NV);
        d.efc_J_rownnz[nefc + r] = NV;
        for (int p = 0; p < NV; p++) d.efc_J_colind[adr0 + (long)r*NV + p] = chain[p];
      }
    }
    double pos[3], off1[3], off2[3], frame[9], fri[5];
    copy3(pos, d.con_pos + 3*i);
    sub3(off1, pos, d.subtree_com + 3*m.body_rootid[b1]);
    sub3(off2, pos, d.subtree_com + 3*m.body_rootid[b2]);
    for (int k = 0; k < 9; k++) frame[k] = d.con_frame[9*i+k];
    for (int k = 0; k < 5; k++) fri[k] = d.con_friction[5*i+k];
    const int rp = dim > 1 ? 3 : 1;
    auto J = d.efc_J + adr0;                // row k's entry p at J[k*NV + p]
    // eight dofs at a time: their loads (chain, cdof) are issued before the chunk's J stores,
    // so each chunk waits once for the stores before it instead of once per dof (the device
    // orders a load after the older stores it cannot prove disjoint)
    constexpr int CH = 8;
    for (int p0 = 0; p0 < NV; p0 += CH) {
      double cj[CH][6];
#pragma unroll
      for (int u = 0; u < CH; u++) {
        for (int r = 0; r < 6; r++) cj[u][r] = 0;
        const int p = p0 + u;
        if (p >= NV) continue;
        const int j = sparse ? chain[p] : p;
        const int bj = m.dof_bodyid[j];
        const bool in1 = ancestorOrSelf(m, bj, b1), in2 = ancestorOrSelf(m, bj, b2);
        if (!(in1 || in2)) continue;
        SP<S> cdof = d.cdof + 6*j;
        // mj_jac rows for this dof (engine_support.c:389-441), zero off the chain
        double jp1[3] = {0, 0, 0}, jp2[3] = {0, 0, 0}, tmp[3];
        if (in1) {
          cross(tmp, cdof, off1);
          jp1[0] = cdof[3] + tmp[0]; jp1[1] = cdof[4] + tmp[1]; jp1[2] = cdof[5] + tmp[2];
        }
        if (in2) {
          cross(tmp, cdof, off2);
          jp2[0] = cdof[3] + tmp[0]; jp2[1] = cdof[4] + tmp[1]; jp2[2] = cdof[5] + tmp[2];
        }
        double jd[3] = {jp2[0] - jp1[0], jp2[1] - jp1[1], jp2[2] - jp1[2]};
        for (int r = 0; r < rp; r++) {
          double acc = 0;
          for (int k = 0; k < 3; k++) {
            double f = frame[3*r+k];
            if (f) acc += jd[k]*f;
          }
          cj[u][r] = acc;
        }
        if (dim > 3) {
          double jr1[3] = {0, 0, 0}, jr2[3] = {0, 0, 0};
          if (in1) { jr1[0] = cdof[0]; jr1[1] = cdof[1]; jr1[2] = cdof[2]; }
          if (in2) { jr2[0] = cdof[0]; jr2[1] = cdof[1]; jr2[2] = cdof[2]; }
          double jdr[3] = {jr2[0] - jr1[0], jr2[1] - jr1[1], jr2[2] - jr1[2]};
          for (int r = 0; r < dim - 3; r++) {
            double acc = 0;
            for (int k = 0; k < 3; k++) {
              double f = frame[3*r+k];
              if (f) acc += jdr[k]*f;
            }
            cj[u][3+r] = acc;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < CH; u++) {
        const int p = p0 + u;
        if (p >= NV) continue;
        if (dim == 1) {
          J[p] = cj[u][0];
        } else if (elliptic) {
          for (int k = 0; k < dim; k++) J[k*NV + p] = cj[u][k];
        } else {
          for (int k = 1; k < dim; k++) {
            double f = fri[k-1];
            J[(2*(k-1))*NV + p] = cj[u][0] + cj[u][k]*f;
            J[(2*(k-1)+1)*NV + p] = cj[u][0] + cj[u][k]*(-f);
          }
        }
      }
    }
    const int type = dim == 1 ? CNSTR_CONTACT_FRICTIONLESS :
                     (elliptic ? CNSTR_CONTACT_ELLIPTIC : CNSTR_CONTACT_PYRAMIDAL);
    for (int r = 0; r < rows; r++) {
      // elliptic rows: pos = (dist, 0, ...), margin = (includemargin, 0, ...) (:1113-1126)
      d.efc_pos[nefc+r] = (elliptic && r) ? 0.0 : d.con_dist[i];
      d.efc_margin[nefc+r] = (elliptic && r) ? 0.0 : d.con_includemargin[i];
      d.efc_frictionloss[nefc+r] = 0;
      d.efc_type[nefc+r] = type;
      d.efc_id[nefc+r] = i;
    }
    rc.nefc = nefc + rows;
  }
}

MJH_HD double dmax(double a, double b) { return a > b ? a : b; }
MJH_HD double dmin(double a, double b) { return a < b ? a : b; }

// getimpedance :1425-1480
MJH_HD void getimpedance(const double* solimp, double pos, double margin, double* imp,
                         double* impP) {
  if (solimp[0] == solimp[1] || solimp[2] <= MINVAL) {
    *imp = 0.5*(solimp[0] + solimp[1]);
    *impP = 0;
    return;
  }
  double x = (pos-margin) / solimp[2];
  double sgn = 1;
  if (x < 0) {
    x = -x;
    sgn = -1;
  }
  if (x >= 1 || x <= 0) {
    *imp = (x >= 1 ? solimp[1] : solimp[0]);
    *impP = 0;
    return;
  }
  double y, yP;
  double p = solimp[4];
  auto power = [](double a, double b) { return b == 1 ? a : (b == 2 ? a*a : pow(a, b)); };
  if (p == 1) {
    y = x;
    yP = 1;
  } else if (x <= solimp[3]) {
    double a = 1/power(solimp[3], p-1);
    y = a*power(x, p);
    yP = p * a*power(x, p-1);
  } else {
    double b = 1/power(1-solimp[3], p-1);
    y = 1-b*power(1-x, p);
    yP = p * b*power(1-x, p-1);
  }
  *imp = solimp[0] + y*(solimp[1]-solimp[0]);
  *impP = yP * sgn * (solimp[1]-solimp[0]) / solimp[2];
}

// mj_makeConstraint :2005-2116 with mj_instantiateFriction (dof, tendon), mj_instantiateLimit
// :824-959 (dense), mj_diagApprox :1138-1311 and mj_makeImpedance :1494-1608 (dim-1 rows)
// CONTACT = false compiles the contact code out (models whose contact capacity is 0); the
// contact path's private arrays would otherwise cost every launch a scratch segment
// getsolparam :1316-1371, the model-side source of a non-contact row's solref/solimp
MJH_HD void rowSolParam(const mjhipModel& m, int tp, int id, double solref[2],
                        double solimp[5]) {
  const double* sr = tp == CNSTR_LIMIT_JOINT ? m.jnt_solref + 2*id :
                     (tp == CNSTR_FRICTION_DOF ? m.dof_solref + 2*id :
                      (tp == CNSTR_EQUALITY ? m.eq_solref + 2*id :
                       (tp == CNSTR_FRICTION_TENDON ? m.tendon_solref_fri + 2*id :
                        m.tendon_solref_lim + 2*id)));
  const double* si = tp == CNSTR_LIMIT_JOINT ? m.jnt_solimp + 5*id :
                     (tp == CNSTR_FRICTION_DOF ? m.dof_solimp + 5*id :
                      (tp == CNSTR_EQUALITY ? m.eq_solimp + 5*id :
                       (tp == CNSTR_FRICTION_TENDON ? m.tendon_solimp_fri + 5*id :
                        m.tendon_solimp_lim + 5*id)));
  solref[0] = sr[0]; solref[1] = sr[1];
  for (int k = 0; k < 5; k++) solimp[k] = si[k];
}

// getsolparam's safety clamps (:1340-1371), then mj_makeImpedance's per-row constants
// (:1494-1560): kbip = (K, B, imp, impP) of a row of type tp at pos/margin
MJH_HD void rowImpedance(const mjhipModel& m, int tp, double* solref, double* solimp,
                         double pos, double margin, double kbip[4]) {
  if ((solref[0] > 0) ^ (solref[1] > 0)) {
    solref[0] = 0.02;
    solref[1] = 1;
  }
  if (!(m.opt.disableflags & mjhipDSBL_REFSAFE) && solref[0] > 0) {
    solref[0] = dmax(solref[0], 2*m.opt.timestep);
  }
  solimp[0] = dmin(mjhipMAXIMP, dmax(mjhipMINIMP, solimp[0]));
  solimp[1] = dmin(mjhipMAXIMP, dmax(mjhipMINIMP, solimp[1]));
  solimp[2] = dmax(0, solimp[2]);
  solimp[3] = dmin(mjhipMAXIMP, dmax(mjhipMINIMP, solimp[3]));
  solimp[4] = dmax(1, solimp[4]);
  double imp, impP;
  getimpedance(solimp, pos, margin, &imp, &impP);
  double K, Bc;
  if (tp == CNSTR_FRICTION_DOF || tp == CNSTR_FRICTION_TENDON) {
    K = 0;
  } else if (solref[0] > 0) {
    K = 1 / dmax(MINVAL, solimp[1]*solimp[1] * solref[0]*solref[0] * solref[1]*solref[1]);
  } else {
    K = -solref[0] / dmax(MINVAL, solimp[1]*solimp[1]);
  }
  if (solref[1] > 0) {
    Bc = 2 / dmax(MINVAL, solimp[1]*solref[0]);
  } else {
    Bc = -solref[1] / dmax(MINVAL, solimp[1]);
  }
  kbip[0] = K;
  kbip[1] = Bc;
  kbip[2] = imp;
  kbip[3] = impP;
}

//---------------------------------- fused constraint rows -----------------------------------
// With skipstage = NONE and no INVDISCRETE, the velocity- and acceleration-stage outputs of a
// row depend only on the row and the inputs qvel, qacc. The fused path therefore finishes
// every row when it is created, in registers: efc_vel and J*qacc in mju_dot's order of
// summation (engine_util_blas.c:680-741), efc_aref (mj_referenceConstraint :2362-2375), force
// and state (mj_constraintUpdate_island :2387-2549 as in invConstraint), and KBIP, R, D and
// diagApprox (mj_diagApprox, mj_makeImpedance). No pass reads back what another pass wrote:
// on the device every such read-back costs a memory round trip per row.
// qfrc_constraint = J'force is one column-blocked pass at the end (constraintForce).

// the remaining outputs of row r from its impedance constants, R and its two dot products
template <int S>
MJH_HD void finishRowFused(const Lane<S>& d, int r, int tp, const double kb[4], double R,
                           double pos, double margin, double frictionloss, double vel,
                           double acc) {
  // outputs no kernel of the call reads back go out as streaming stores
  for (int k = 0; k < 4; k++) MJH_NT_STORE(d.efc_KBIP[4*r+k], kb[k]);
  const double D = 1 / R;
  MJH_NT_STORE(d.efc_R[r], R);
  MJH_NT_STORE(d.efc_D[r], D);
  MJH_NT_STORE(d.efc_diagApprox[r], R * kb[2] / (1-kb[2]));
  MJH_NT_STORE(d.efc_vel[r], vel);
  const double aref = -kb[1]*vel - kb[0]*kb[2]*(pos-margin);
  MJH_NT_STORE(d.efc_aref[r], aref);
  const double jar = acc - aref;
  MJH_NT_STORE(d.jar[r], jar);
  double force = -D * jar;
  int state = CNSTRSTATE_QUADRATIC;
  if (tp == CNSTR_FRICTION_DOF || tp == CNSTR_FRICTION_TENDON) {
    const double Rf = R * frictionloss;
    if (jar <= -Rf) {
      force = frictionloss;
      state = CNSTRSTATE_LINEARNEG;
    } else if (jar >= Rf) {
      force = -frictionloss;
      state = CNSTRSTATE_LINEARPOS;
    }
  } else if (tp != CNSTR_EQUALITY && jar >= 0) {
    force = 0;
    state = CNSTRSTATE_SATISFIED;
  }
  d.efc_force[r] = force;
  if (d.fst && r < d.nfst) d.fst[r] = force;
  d.efc_state[r] = state;
}

// a friction or limit row just added at r (few per instance: its J row is read back)
// (vel, acc = J*qvel, J*qacc of the row, already formed)
template <int S>
MJH_HD void finishNonContactVA(const mjhipModel& m, const Lane<S>& d, int r, int tp, int id,
                               double pos, double margin, double frictionloss, double vel,
                               double acc) {
  const double diag = tp == CNSTR_FRICTION_DOF ? m.dof_invweight0[id] :
                      (tp == CNSTR_LIMIT_JOINT ? m.dof_invweight0[m.jnt_dofadr[id]] :
                       m.tendon_invweight0[id]);
  double solref[2], solimp[5], kb[4];
  rowSolParam(m, tp, id, solref, solimp);
  rowImpedance(m, tp, solref, solimp, pos, margin, kb);
  const double R = dmax(MINVAL, (1-kb[2])*diag/kb[2]);
  finishRowFused(d, r, tp, kb, R, pos, margin, frictionloss, vel, acc);
}

template <int S>
MJH_HD void finishNonContact(const mjhipModel& m, const Lane<S>& d, int r, int tp, int id,
                             double pos, double margin, double frictionloss) {
  auto J = d.efc_J + r*m.nv;
  finishNonContactVA(m, d, r, tp, id, pos, margin, frictionloss, dot(J, d.qvel, m.nv),
                     dot(J, d.qacc, m.nv));
}

// indexable views for dot(): a generator of row values, and a strided (LDS) column
template <class F>
struct FnIdx {
  F f;
  MJH_HD double operator[](int k) const { return f(k); }
};
template <int STRIDE>
struct StridedIdx {
  const double* p;
  MJH_HD double operator[](int k) const { return p[k*STRIDE]; }
};

// One contact's rows (condim DIM) at efc row `nefc`. As instantiateContact, the rows are
// formed dof by dof straight into efc_J, here in blocks of four dofs whose loads (cdof,
// qvel, qacc) are issued together. The chain test is a bit test of chain masks. For DIM <= 3
// J*qvel and J*qacc accumulate in registers in mju_dot's four partial sums; wider contacts
// read their rows back. All rows of a contact share K, B, imp, impP and R (mj_makeImpedance:
// one impedance per contact; pyramidal R is 2 mu^2 R0 for every row, :1562-1598).
template <int S, int DIM>
MJH_HD void contactRowsFused(const mjhipModel& m, const Lane<S>& d, int i, int nefc) {
  constexpr int ROWS = DIM == 1 ? 1 : 2*(DIM - 1);
  constexpr bool REG = DIM <= 3;
  constexpr int NA = REG ? ROWS : 1;
  const int nv = m.nv;
  const int tp = DIM == 1 ? CNSTR_CONTACT_FRICTIONLESS : CNSTR_CONTACT_PYRAMIDAL;
  MJH_TICK(tc0);
  int b1, b2, rt1, rt2;
  if (d.cbody && i < d.ncbody) {
    b1 = d.cbody[4*i];
    b2 = d.cbody[4*i+1];
    rt1 = d.cbody[4*i+2];
    rt2 = d.cbody[4*i+3];
  } else {
    b1 = m.geom_bodyid[d.con_geom[2*i]];
    b2 = m.geom_bodyid[d.con_geom[2*i+1]];
    rt1 = m.body_rootid[b1];
    rt2 = m.body_rootid[b2];
  }
  double pos[3], frame[9], fri[5], solref[2], solimp[5];
  for (int k = 0; k < 3; k++) pos[k] = d.con_pos[3*i+k];
  for (int k = 0; k < 9; k++) frame[k] = d.con_frame[9*i+k];
  for (int k = 0; k < 5; k++) fri[k] = d.con_friction[5*i+k];
  for (int k = 0; k < 2; k++) solref[k] = d.con_solref[2*i+k];
  for (int k = 0; k < 5; k++) solimp[k] = d.con_solimp[5*i+k];
  const double dist = d.con_dist[i], incl = d.con_includemargin[i];
  double off1[3], off2[3];
  sub3(off1, pos, d.subtree_com + 3*rt1);
  sub3(off2, pos, d.subtree_com + 3*rt2);
  const unsigned long long mask1 = d.chain[b1], mask2 = d.chain[b2];

  // impedance and R (mj_diagApprox :1138-1311 with mj_makeImpedance)
  double kb[4];
  rowImpedance(m, tp, solref, solimp, dist, incl, kb);
  double tran = 0, rot = 0;
  tran += m.body_invweight0[2*b1] * 1.0;
  rot += m.body_invweight0[2*b1+1] * 1.0;
  tran += m.body_invweight0[2*b2] * 1.0;
  rot += m.body_invweight0[2*b2+1] * 1.0;
  (void)rot;
  double R;
  if constexpr (DIM == 1) {
    R = dmax(MINVAL, (1-kb[2])*tran/kb[2]);
  } else {
    const double v0 = tran + fri[0]*fri[0]*tran;
    const double R0 = dmax(MINVAL, (1-kb[2])*v0/kb[2]);
    const double R1 = R0/dmax(MINVAL, m.opt.impratio);
    const double mu = fri[0] * sqrt(R1/R0);
    d.con_mu[i] = mu;
    R = 2*mu*mu*R0;
  }

  MJH_TICK(tc1);
  // rows, dof by dof, in blocks of four
  auto J = d.efc_J + nefc*nv;
  double av[NA][4], aa[NA][4], tv[NA], ta[NA];
  for (int r = 0; r < NA; r++) {
    for (int k = 0; k < 4; k++) av[r][k] = aa[r][k] = 0;
    tv[r] = ta[r] = 0;
  }
  const int nb4 = (nv / 4) * 4;
  constexpr int BLK = REG ? 4 : 1;   // wide contacts (rare) go one dof at a time
  for (int jb = 0; jb < nv; jb += BLK) {
    const bool full = jb + 4 <= nv;
    double cd[BLK][6], qv[BLK], qa[BLK];
#pragma unroll
    for (int k = 0; k < BLK; k++) {
      const int j = jb + k;
      if (j < nv && d.cdq) {            // the cooperative kernel's LDS copy
        const double* p = d.cdq + 8*j;
        for (int c = 0; c < 6; c++) cd[k][c] = p[c];
        if constexpr (REG) {
          qv[k] = p[6];
          qa[k] = p[7];
        }
      } else if (j < nv) {
        for (int c = 0; c < 6; c++) cd[k][c] = d.cdof[6*j+c];
        if constexpr (REG) {
          qv[k] = d.qvel[j];
          qa[k] = d.qacc[j];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < BLK; k++) {
      const int j = jb + k;
      if (j >= nv) break;
      const int bj = m.dof_bodyid[j];
      const bool in1 = (mask1 >> bj) & 1, in2 = (mask2 >> bj) & 1;
      // mj_jac rows for this dof (engine_support.c:389-441), zero off the chain
      double t1[3], t2[3], jd[3], cj[6] = {0, 0, 0, 0, 0, 0};
      cross(t1, cd[k], off1);
      cross(t2, cd[k], off2);
      for (int c = 0; c < 3; c++) {
        const double p1 = in1 ? cd[k][3+c] + t1[c] : 0.0;
        const double p2 = in2 ? cd[k][3+c] + t2[c] : 0.0;
        jd[c] = p2 - p1;
      }
      const int rp = DIM > 1 ? 3 : 1;
      for (int r = 0; r < rp; r++) {
        double acc = 0;
        for (int c = 0; c < 3; c++) {
          const double f = frame[3*r+c];
          if (f) acc += jd[c]*f;
        }
        cj[r] = acc;
      }
      if constexpr (DIM > 3) {
        double jdr[3];
        for (int c = 0; c < 3; c++) jdr[c] = (in2 ? cd[k][c] : 0.0) - (in1 ? cd[k][c] : 0.0);
        for (int r = 0; r < DIM - 3; r++) {
          double acc = 0;
          for (int c = 0; c < 3; c++) {
            const double f = frame[3*r+c];
            if (f) acc += jdr[c]*f;
          }
          cj[3+r] = acc;
        }
      }
      double Jv[ROWS];
      if constexpr (DIM == 1) {
        Jv[0] = cj[0];
      } else {
        for (int c = 1; c < DIM; c++) {
          const double f = fri[c-1];
          Jv[2*(c-1)] = cj[0] + cj[c]*f;
          Jv[2*(c-1)+1] = cj[0] + cj[c]*(-f);
        }
      }
      for (int r = 0; r < ROWS; r++) J[r*nv + j] = Jv[r];
      if constexpr (REG) {
        for (int r = 0; r < ROWS; r++) {
          const double pv = Jv[r]*qv[k], pa = Jv[r]*qa[k];
          if (full) {
            av[r][k] += pv;
            aa[r][k] += pa;
          } else {
            tv[r] = j == nb4 ? pv : tv[r] + pv;
            ta[r] = j == nb4 ? pa : ta[r] + pa;
          }
        }
      }
    }
  }
  MJH_TICK(tc2);
  for (int r = 0; r < ROWS; r++) {
    double vel, acc;
    if constexpr (REG) {
      vel = (av[r][0] + av[r][2]) + (av[r][1] + av[r][3]);
      acc = (aa[r][0] + aa[r][2]) + (aa[r][1] + aa[r][3]);
      if (nv > nb4) {
        vel += tv[r];
        acc += ta[r];
      }
    } else {
      vel = dot(J + r*nv, d.qvel, nv);
      acc = dot(J + r*nv, d.qacc, nv);
    }
    const int row = nefc + r;
    d.efc_pos[row] = dist;
    d.efc_margin[row] = incl;
    d.efc_frictionloss[row] = 0;
    d.efc_type[row] = tp;
    d.efc_id[row] = i;
    finishRowFused(d, row, tp, kb, R, dist, incl, 0, vel, acc);
  }
  MJH_TICK(tc3);
  MJH_SPAN(0, tc0, tc1);        // contact data, impedance, R
  MJH_SPAN(2, tc1, tc2);        // the dof loop
  MJH_SPAN(4, tc2, tc3);        // row fields and finish
}

#if defined(__HIPCC__)   // wave shuffles: HIP builds only (the host harness has no lanes)
// contactRowsFused for a frictionless or condim-3 pyramidal contact split over Q lanes (the
// cooperative constraint kernel; q = this lane's index in the contact's lane group, the group
// aligned to Q in the wave). Lane q forms the dofs j of the four-dof blocks with j % 4 = q
// (mod Q): exactly mju_dot's partial sums res0..res3 (engine_util_blas.c:720-729) for
// J*qvel and J*qacc, which two shuffle steps then combine as (res0 + res2) + (res1 + res3);
// lane 0 adds the tail (:733-741). Lane q finishes rows r % Q = q. Every value equals
// contactRowsFused's.
template <int S, int DIM, int Q>
MJH_HD void contactRowsSplit(const mjhipModel& m, const Lane<S>& d, int i, int nefc, int q) {
  static_assert(DIM == 1 || DIM == 3, "wide contacts keep one lane");
  static_assert(Q == 1 || Q == 2 || Q == 4, "a divisor of mju_dot's four partial sums");
  constexpr int ROWS = DIM == 1 ? 1 : 4;
  constexpr int T = 4 / Q;                 // partial sums per lane: k = q + Q t
  const int nv = m.nv;
  const int tp = DIM == 1 ? CNSTR_CONTACT_FRICTIONLESS : CNSTR_CONTACT_PYRAMIDAL;
  int b1, b2, rt1, rt2;
  if (d.cbody && i < d.ncbody) {
    b1 = d.cbody[4*i];
    b2 = d.cbody[4*i+1];
    rt1 = d.cbody[4*i+2];
    rt2 = d.cbody[4*i+3];
  } else {
    b1 = m.geom_bodyid[d.con_geom[2*i]];
    b2 = m.geom_bodyid[d.con_geom[2*i+1]];
    rt1 = m.body_rootid[b1];
    rt2 = m.body_rootid[b2];
  }
  double pos[3], frame[9], fri[5], solref[2], solimp[5];
  for (int k = 0; k < 3; k++) pos[k] = d.con_pos[3*i+k];
  for (int k = 0; k < 9; k++) frame[k] = d.con_frame[9*i+k];
  for (int k = 0; k < 5; k++) fri[k] = d.con_friction[5*i+k];
  for (int k = 0; k < 2; k++) solref[k] = d.con_solref[2*i+k];
  for (int k = 0; k < 5; k++) solimp[k] = d.con_solimp[5*i+k];
  const double dist = d.con_dist[i], incl = d.con_includemargin[i];
  double off1[3], off2[3];
  sub3(off1, pos, d.subtree_com + 3*rt1);
  sub3(off2, pos, d.subtree_com + 3*rt2);
  // the dofs on each body's chain (d.dchain, the kernel's LDS table): a bit test per dof. The
  // dof is lane-dependent here, so reading its body id from memory would be a vector load,
  // and every vector load waits for the lane's earlier row stores.
  const unsigned long long mask1 = d.dchain[b1], mask2 = d.dchain[b2];
  double kb[4];
  rowImpedance(m, tp, solref, solimp, dist, incl, kb);
  double tran = 0;
  tran += m.body_invweight0[2*b1] * 1.0;
  tran += m.body_invweight0[2*b2] * 1.0;
  double R;
  if constexpr (DIM == 1) {
    R = dmax(MINVAL, (1-kb[2])*tran/kb[2]);
  } else {
    const double v0 = tran + fri[0]*fri[0]*tran;
    const double R0 = dmax(MINVAL, (1-kb[2])*v0/kb[2]);
    const double R1 = R0/dmax(MINVAL, m.opt.impratio);
    const double mu = fri[0] * sqrt(R1/R0);
    if (q == 0) d.con_mu[i] = mu;
    R = 2*mu*mu*R0;
  }

  auto J = d.efc_J + nefc*nv;
  // one dof's rows into efc_J, returned in Jv (as contactRowsFused forms them)
  auto dofRows = [&](int j, const double* cd, double Jv[ROWS]) MJH_LAMBDA_INLINE {
    const bool in1 = (mask1 >> j) & 1, in2 = (mask2 >> j) & 1;
    double t1[3], t2[3], jd[3], cj[3] = {0, 0, 0};
    cross(t1, cd, off1);
    cross(t2, cd, off2);
    for (int c = 0; c < 3; c++) {
      const double p1 = in1 ? cd[3+c] + t1[c] : 0.0;
      const double p2 = in2 ? cd[3+c] + t2[c] : 0.0;
      jd[c] = p2 - p1;
    }
    constexpr int rp = DIM > 1 ? 3 : 1;
    for (int r = 0; r < rp; r++) {
      double acc = 0;
      for (int c = 0; c < 3; c++) {
        const double f = frame[3*r+c];
        if (f) acc += jd[c]*f;
      }
      cj[r] = acc;
    }
    if constexpr (DIM == 1) {
      Jv[0] = cj[0];
    } else {
      for (int c = 1; c < 3; c++) {
        const double f = fri[c-1];
        Jv[2*(c-1)] = cj[0] + cj[c]*f;
        Jv[2*(c-1)+1] = cj[0] + cj[c]*(-f);
      }
    }
    for (int r = 0; r < ROWS; r++) J[r*nv + j] = Jv[r];
  };
  double av[ROWS][T], aa[ROWS][T], tv[ROWS], ta[ROWS];
  for (int r = 0; r < ROWS; r++) {
    for (int t = 0; t < T; t++) av[r][t] = aa[r][t] = 0;
    tv[r] = ta[r] = 0;
  }
  const int nb4 = (nv / 4) * 4;
  for (int jb = 0; jb < nb4; jb += 4) {
    double cd[T][6], qv[T], qa[T];
#pragma unroll
    for (int t = 0; t < T; t++) {
      const double* p = d.cdq + 8*(jb + q + Q*t);
      for (int c = 0; c < 6; c++) cd[t][c] = p[c];
      qv[t] = p[6];
      qa[t] = p[7];
    }
#pragma unroll
    for (int t = 0; t < T; t++) {
      double Jv[ROWS];
      dofRows(jb + q + Q*t, cd[t], Jv);
      for (int r = 0; r < ROWS; r++) {
        av[r][t] += Jv[r]*qv[t];
        aa[r][t] += Jv[r]*qa[t];
      }
    }
  }
  if (q == 0) {                           // the tail dofs, summed on their own (:733-741)
    for (int j = nb4; j < nv; j++) {
      const double* p = d.cdq + 8*j;
      double cd[6], Jv[ROWS];
      for (int c = 0; c < 6; c++) cd[c] = p[c];
      dofRows(j, cd, Jv);
      for (int r = 0; r < ROWS; r++) {
        const double pv = Jv[r]*p[6], pa = Jv[r]*p[7];
        tv[r] = j == nb4 ? pv : tv[r] + pv;
        ta[r] = j == nb4 ? pa : ta[r] + pa;
      }
    }
  }
  for (int r = 0; r < ROWS; r++) {
    // (res0 + res2) + (res1 + res3): addition commutes exactly, so each lane may add its
    // partner's partial to its own
    double sv, sa;
    if constexpr (Q == 4) {
      sv = av[r][0] + __shfl_xor(av[r][0], 2, 4);
      sa = aa[r][0] + __shfl_xor(aa[r][0], 2, 4);
      sv = sv + __shfl_xor(sv, 1, 4);
      sa = sa + __shfl_xor(sa, 1, 4);
    } else if constexpr (Q == 2) {
      sv = av[r][0] + av[r][1];
      sa = aa[r][0] + aa[r][1];
      sv = sv + __shfl_xor(sv, 1, 2);
      sa = sa + __shfl_xor(sa, 1, 2);
    } else {
      sv = (av[r][0] + av[r][2]) + (av[r][1] + av[r][3]);
      sa = (aa[r][0] + aa[r][2]) + (aa[r][1] + aa[r][3]);
    }
    if (nv > nb4) {
      sv += Q > 1 ? __shfl(tv[r], 0, Q) : tv[r];
      sa += Q > 1 ? __shfl(ta[r], 0, Q) : ta[r];
    }
    if (r % Q != q) continue;
    const int row = nefc + r;
    d.efc_pos[row] = dist;
    d.efc_margin[row] = incl;
    d.efc_frictionloss[row] = 0;
    d.efc_type[row] = tp;
    d.efc_id[row] = i;
    finishRowFused(d, row, tp, kb, R, dist, incl, 0, sv, sa);
  }
}
#endif

// mj_instantiateContact :964-1131 on the fused path (pyramidal or frictionless)
template <int S>
MJH_HD void instantiateContactFused(const mjhipModel& m, const Lane<S>& d, RowCount& rc,
                                    int* status) {
  const int ncon = d.con_count[0];
  if ((m.opt.disableflags & mjhipDSBL_CONTACT) || ncon == 0 || m.nv == 0) return;
  for (int i = 0; i < ncon; i++) {
    if (d.con_exclude[i]) continue;
    const int dim = d.con_dim[i];
    const int rows = dim == 1 ? 1 : 2*(dim - 1);
    d.con_efc_address[i] = rc.nefc;
    if (rc.nefc + rows > d.efc_cap) {   // mjWARN_CNSTRFULL analogue (capacity is exact)
      *status |= MJHIP_INST_CNSTRFULL;
      continue;
    }
    switch (dim) {
      case 1: contactRowsFused<S, 1>(m, d, i, rc.nefc); break;
      case 3: contactRowsFused<S, 3>(m, d, i, rc.nefc); break;
      case 4: contactRowsFused<S, 4>(m, d, i, rc.nefc); break;
      default: contactRowsFused<S, 6>(m, d, i, rc.nefc); break;
    }
    rc.nefc += rows;
  }
}

// qfrc_constraint = J'force (mju_mulMatTVec engine_util_blas.c:756-766: rows in order, zero
// forces skipped) in blocks of 8 columns x 4 rows: 36 independent loads per step
template <int S>
MJH_HD void constraintForce(const mjhipModel& m, const Lane<S>& d, int nefc) {
  const int nv = m.nv;
  for (int c0 = 0; c0 < nv; c0 += 8) {
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int r = 0;
    for (; r + 4 <= nefc; r += 4) {
      double f[4], Jv[4][8];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        f[k] = d.efc_force[r+k];
        for (int c = 0; c < 8; c++) Jv[k][c] = c0 + c < nv ? d.efc_J[(r+k)*nv + c0 + c] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (f[k]) {
          for (int c = 0; c < 8; c++) acc[c] += Jv[k][c]*f[k];
        }
      }
    }
    for (; r < nefc; r++) {
      const double f = d.efc_force[r];
      if (f) {
        for (int c = 0; c < 8; c++) {
          if (c0 + c < nv) acc[c] += d.efc_J[r*nv + c0 + c]*f;
        }
      }
    }
    for (int c = 0; c < 8; c++) {
      if (c0 + c < nv) d.qfrc_constraint[c0 + c] = acc[c];
    }
  }
}

// mju_mulQuatAxis engine_util_spatial.c:81-92
template <class A> MJH_HD void mulQuatAxis(double res[4], const double q[4], A axis) {
  const double t0 = -q[1]*axis[0] - q[2]*axis[1] - q[3]*axis[2];
  const double t1 = q[0]*axis[0] + q[2]*axis[2] - q[3]*axis[1];
  const double t2 = q[0]*axis[1] + q[3]*axis[0] - q[1]*axis[2];
  const double t3 = q[0]*axis[2] + q[1]*axis[1] - q[2]*axis[0];
  res[0] = t0; res[1] = t1; res[2] = t2; res[3] = t3;
}

// diagApprox of equality row k (0-based within its constraint) of equality `id`
// (mj_diagApprox :1151-1197; a weld's rows 0-2 are translational, 3-5 rotational)
MJH_HD double eqDiagApprox(const mjhipModel& m, int id, int k) {
  const int t = m.eq_type[id];
  if (t == mjhipEQ_CONNECT || t == mjhipEQ_WELD) {
    int b1 = m.eq_obj1id[id], b2 = m.eq_obj2id[id];
    if (m.eq_objtype[id] == 6) {
      b1 = m.site_bodyid[b1];
      b2 = m.site_bodyid[b2];
    }
    const int r = (t == mjhipEQ_WELD && k > 2) ? 1 : 0;
    return m.body_invweight0[2*b1 + r] + m.body_invweight0[2*b2 + r];
  }
  double dA = t == mjhipEQ_JOINT ? m.dof_invweight0[m.jnt_dofadr[m.eq_obj1id[id]]] :
                                   m.tendon_invweight0[m.eq_obj1id[id]];
  if (m.eq_obj2id[id] >= 0) {
    dA += t == mjhipEQ_JOINT ? m.dof_invweight0[m.jnt_dofadr[m.eq_obj2id[id]]] :
                               m.tendon_invweight0[m.eq_obj2id[id]];
  }
  return dA;
}

// mj_instantiateEquality :493-764 (dense; connect, weld, joint, tendon; eq_active0). The
// rows are formed dof by dof straight into efc_J: the two body Jacobians of mj_jacDifPair
// (dense: mj_jac twice, then jac2 - jac1) are zero off their chains, and every other step
// (the weld's rotational correction and torquescale) acts column by column.
template <int S>
MJH_HD void instantiateEqualitySparse(const mjhipModel& m, const Lane<S>& d, RowCount& rc,
                                      int* status);

template <int S, bool FUSED>
MJH_HD void instantiateEquality(const mjhipModel& m, const Lane<S>& d, RowCount& rc,
                                int* status) {
  const int nv = m.nv;
  if ((m.opt.disableflags & mjhipDSBL_EQUALITY) || m.neq == 0) return;
  if (!FUSED && mjh_isSparse(&m)) {
    instantiateEqualitySparse(m, d, rc, status);
    return;
  }
  for (int i = 0; i < m.neq; i++) {
    if (!m.eq_active0[i]) continue;
    const double* data = m.eq_data + mjhipNEQDATA*i;
    const int t = m.eq_type[i];
    const int id0 = m.eq_obj1id[i], id1 = m.eq_obj2id[i];
    const int size = t == mjhipEQ_CONNECT ? 3 : (t == mjhipEQ_WELD ? 6 : 1);
    const int r0 = rc.nefc;
    if (r0 + size > d.efc_cap) {
      *status |= MJHIP_INST_CNSTRFULL;
      continue;
    }
    auto J = d.efc_J + r0*nv;
    double cpos[6];
    if (t == mjhipEQ_CONNECT || t == mjhipEQ_WELD) {
      double pos[2][3];
      int body[2];
      const int ids[2] = {id0, id1};
      for (int j = 0; j < 2; j++) {
        if (m.eq_objtype[i] == 1) {
          const double* anchor = data + 3*(t == mjhipEQ_WELD ? 1 - j : j);
          mulMatVec3(pos[j], d.xmat + 9*ids[j], anchor);
          addTo3(pos[j], d.xpos + 3*ids[j]);
          body[j] = ids[j];
        } else {
          copy3(pos[j], d.site_xpos + 3*ids[j]);
          body[j] = m.site_bodyid[ids[j]];
        }
      }
      sub3(cpos, pos[0], pos[1]);
      double off0[3], off1[3];
      sub3(off0, pos[0], d.subtree_com + 3*m.body_rootid[body[0]]);
      sub3(off1, pos[1], d.subtree_com + 3*m.body_rootid[body[1]]);
      double quat[4], quat1[4], torquescale = 0;
      if (t == mjhipEQ_WELD) {
        torquescale = data[10];
        if (m.eq_objtype[i] == 1) {
          mulQuat(quat, d.xquat + 4*id0, data + 6);
          copy4(quat1, d.xquat + 4*id1);
        } else {
          mulQuat(quat, d.xquat + 4*body[0], m.site_quat + 4*id0);
          mulQuat(quat1, d.xquat + 4*body[1], m.site_quat + 4*id1);
        }
        quat1[1] = -quat1[1]; quat1[2] = -quat1[2]; quat1[3] = -quat1[3];
        double quat2[4];
        mulQuat(quat2, quat1, quat);
        cpos[3] = quat2[1]*torquescale;
        cpos[4] = quat2[2]*torquescale;
        cpos[5] = quat2[3]*torquescale;
      }
      for (int j = 0; j < nv; j++) {
        const int bj = m.dof_bodyid[j];
        const bool in0 = ancestorOrSelf(m, bj, body[0]), in1 = ancestorOrSelf(m, bj, body[1]);
        double jp0[3] = {0, 0, 0}, jp1[3] = {0, 0, 0}, jr0[3] = {0, 0, 0}, jr1[3] = {0, 0, 0};
        SP<S> cdof = d.cdof + 6*j;
        double tmp[3];
        if (in0) {
          cross(tmp, cdof, off0);
          jp0[0] = cdof[3] + tmp[0]; jp0[1] = cdof[4] + tmp[1]; jp0[2] = cdof[5] + tmp[2];
          jr0[0] = cdof[0]; jr0[1] = cdof[1]; jr0[2] = cdof[2];
        }
        if (in1) {
          cross(tmp, cdof, off1);
          jp1[0] = cdof[3] + tmp[0]; jp1[1] = cdof[4] + tmp[1]; jp1[2] = cdof[5] + tmp[2];
          jr1[0] = cdof[0]; jr1[1] = cdof[1]; jr1[2] = cdof[2];
        }
        for (int k = 0; k < 3; k++) J[k*nv + j] = jp0[k] - jp1[k];
        if (t == mjhipEQ_WELD) {
          double axis[3] = {jr0[0] - jr1[0], jr0[1] - jr1[1], jr0[2] - jr1[2]};
          double quat2[4], quat3[4];
          mulQuatAxis(quat2, quat1, axis);
          mulQuat(quat3, quat2, quat);
          for (int k = 0; k < 3; k++) J[(3 + k)*nv + j] = (0.5*quat3[1 + k])*torquescale;
        }
      }
    } else {
      // joint / tendon coupling with a quartic polynomial
      double p0, ref0;
      if (t == mjhipEQ_JOINT) {
        p0 = d.qpos[m.jnt_qposadr[id0]];
        ref0 = m.qpos0[m.jnt_qposadr[id0]];
        zero(J, nv);
        J[m.jnt_dofadr[id0]] = 1;
      } else {
        p0 = d.ten_length[id0];
        ref0 = m.tendon_length0[id0];
        copy(J, d.ten_J + id0*nv, nv);
      }
      if (id1 >= 0) {
        double p1, ref1;
        if (t == mjhipEQ_JOINT) {
          p1 = d.qpos[m.jnt_qposadr[id1]];
          ref1 = m.qpos0[m.jnt_qposadr[id1]];
        } else {
          p1 = d.ten_length[id1];
          ref1 = m.tendon_length0[id1];
        }
        const double dif = p1 - ref1;
        cpos[0] = p0 - ref0 - data[0] -
                  (data[1]*dif + data[2]*dif*dif + data[3]*dif*dif*dif + data[4]*dif*dif*dif*dif);
        const double deriv = data[1] + 2*data[2]*dif + 3*data[3]*dif*dif +
                             4*data[4]*dif*dif*dif;
        if (t == mjhipEQ_JOINT) {
          const int c = m.jnt_dofadr[id1];
          J[c] = J[c] + 1*-deriv;
        } else {
          addToScl(J, d.ten_J + id1*nv, -deriv, nv);
        }
      } else {
        cpos[0] = p0 - ref0 - data[0];
      }
    }
    // mj_addConstraint: an all-zero Jacobian adds no rows
    bool empty = true;
    for (int k = 0; empty && k < size*nv; k++) empty = J[k] == 0;
    if (empty) continue;
    for (int k = 0; k < size; k++) {
      d.efc_pos[r0+k] = cpos[k];
      d.efc_margin[r0+k] = 0;
      d.efc_frictionloss[r0+k] = 0;
      d.efc_type[r0+k] = CNSTR_EQUALITY;
      d.efc_id[r0+k] = i;
    }
    rc.nefc += size;
    rc.ne += size;
    if constexpr (FUSED) {
      // getposdim :1392-1422: connect/weld rows share the impedance of the block's norm
      const double ipos = size > 1 ? sqrt(dot(cpos, cpos, size)) : cpos[0];
      double solref[2], solimp[5], kb[4];
      rowSolParam(m, CNSTR_EQUALITY, i, solref, solimp);
      rowImpedance(m, CNSTR_EQUALITY, solref, solimp, ipos, 0, kb);
      for (int k = 0; k < size; k++) {
        const double R = dmax(MINVAL, (1-kb[2])*eqDiagApprox(m, i, k)/kb[2]);
        const auto Jr = J + k*nv;
        finishRowFused(d, r0 + k, CNSTR_EQUALITY, kb, R, cpos[k], 0, 0, dot(Jr, d.qvel, nv),
                       dot(Jr, d.qacc, nv));
      }
    }
  }
}

// mj_instantiateEquality :493-764, sparse branch: connect and weld rows over the merged chain
// of the two bodies (mj_jacDifPair), joint and tendon couplings over the objects' chains
// combined by mju_combineSparse (:702-707); the values are the dense rows' at the chain's dofs
template <int S>
MJH_HD void instantiateEqualitySparse(const mjhipModel& m, const Lane<S>& d, RowCount& rc,
                                      int* status) {
  const int nv = m.nv;
  SP<S, int> chain = d.chainbuf, chain2 = d.chainbuf + nv, bufind = d.chainbuf + 2*nv;
  for (int i = 0; i < m.neq; i++) {
    if (!m.eq_active0[i]) continue;
    const double* data = m.eq_data + mjhipNEQDATA*i;
    const int t = m.eq_type[i];
    const int id0 = m.eq_obj1id[i], id1 = m.eq_obj2id[i];
    double cpos[6];
    if (t == mjhipEQ_CONNECT || t == mjhipEQ_WELD) {
      const int size = t == mjhipEQ_CONNECT ? 3 : 6;
      double pos[2][3];
      int body[2];
      const int ids[2] = {id0, id1};
      for (int j = 0; j < 2; j++) {
        if (m.eq_objtype[i] == 1) {
          const double* anchor = data + 3*(t == mjhipEQ_WELD ? 1 - j : j);
          mulMatVec3(pos[j], d.xmat + 9*ids[j], anchor);
          addTo3(pos[j], d.xpos + 3*ids[j]);
          body[j] = ids[j];
        } else {
          copy3(pos[j], d.site_xpos + 3*ids[j]);
          body[j] = m.site_bodyid[ids[j]];
        }
      }
      sub3(cpos, pos[0], pos[1]);
      double off0[3], off1[3];
      sub3(off0, pos[0], d.subtree_com + 3*m.body_rootid[body[0]]);
      sub3(off1, pos[1], d.subtree_com + 3*m.body_rootid[body[1]]);
      double quat[4], quat1[4], torquescale = 0;
      if (t == mjhipEQ_WELD) {
        torquescale = data[10];
        if (m.eq_objtype[i] == 1) {
          mulQuat(quat, d.xquat + 4*id0, data + 6);
          copy4(quat1, d.xquat + 4*id1);
        } else {
          mulQuat(quat, d.xquat + 4*body[0], m.site_quat + 4*id0);
          mulQuat(quat1, d.xquat + 4*body[1], m.site_quat + 4*id1);
        }
        quat1[1] = -quat1[1]; quat1[2] = -quat1[2]; quat1[3] = -quat1[3];
        double quat2[4];
        mulQuat(quat2, quat1, quat);
        cpos[3] = quat2[1]*torquescale;
        cpos[4] = quat2[2]*torquescale;
        cpos[5] = quat2[3]*torquescale;
      }
      const int NV = mergeChain(m, chain, body[1], body[0]);
      if (!NV) continue;                   // mj_addConstraint: empty chain, no rows
      const int r0 = rc.nefc;
      const long adr0 = r0 ? d.efc_J_rowadr[r0-1] + d.efc_J_rownnz[r0-1] : 0;
      if (r0 + size > d.efc_cap || adr0 + (long)size*NV > d.nj_cap) {
        *status |= MJHIP_INST_CNSTRFULL;
        continue;
      }
      auto J = d.efc_J + adr0;
      for (int p = 0; p < NV; p++) {
        const int j = chain[p];
        const int bj = m.dof_bodyid[j];
        const bool in0 = ancestorOrSelf(m, bj, body[0]), in1 = ancestorOrSelf(m, bj, body[1]);
        double jp0[3] = {0, 0, 0}, jp1[3] = {0, 0, 0}, jr0[3] = {0, 0, 0}, jr1[3] = {0, 0, 0};
        SP<S> cdof = d.cdof + 6*j;
        double tmp[3];
        if (in0) {
          cross(tmp, cdof, off0);
          jp0[0] = cdof[3] + tmp[0]; jp0[1] = cdof[4] + tmp[1]; jp0[2] = cdof[5] + tmp[2];
          jr0[0] = cdof[0]; jr0[1] = cdof[1]; jr0[2] = cdof[2];
        }
        if (in1) {
          cross(tmp, cdof, off1);
          jp1[0] = cdof[3] + tmp[0]; jp1[1] = cdof[4] + tmp[1]; jp1[2] = cdof[5] + tmp[2];
          jr1[0] = cdof[0]; jr1[1] = cdof[1]; jr1[2] = cdof[2];
        }
        for (int k = 0; k < 3; k++) J[k*NV + p] = jp0[k] - jp1[k];
        if (t == mjhipEQ_WELD) {
          double axis[3] = {jr0[0] - jr1[0], jr0[1] - jr1[1], jr0[2] - jr1[2]};
          double quat2[4], quat3[4];
          mulQuatAxis(quat2, quat1, axis);
          mulQuat(quat3, quat2, quat);
          for (int k = 0; k < 3; k++) J[(3 + k)*NV + p] = (0.5*quat3[1 + k])*torquescale;
        }
      }
      for (int k = 0; k < size; k++) {
        d.efc_J_rowadr[r0+k] = (int)(adr0 + (long)k*NV);
        d.efc_J_rownnz[r0+k] = NV;
        for (int p = 0; p < NV; p++) d.efc_J_colind[adr0 + (long)k*NV + p] = chain[p];
        d.efc_pos[r0+k] = cpos[k];
        d.efc_margin[r0+k] = 0;
        d.efc_frictionloss[r0+k] = 0;
        d.efc_type[r0+k] = CNSTR_EQUALITY;
        d.efc_id[r0+k] = i;
      }
      rc.nefc += size;
      rc.ne += size;
      continue;
    }
    // joint / tendon coupling: the first object's row in jacp[0, nv), the second's in
    // jacp[nv, 2nv), combined into the first
    SP<S> jac0 = d.jacp, jac1 = d.jacp + nv;
    int NV = 0, NV2 = 0;
    double pv[2], ref[2];
    const int ids[2] = {id0, id1};
    for (int j = 0; j < 1 + (id1 >= 0); j++) {
      SP<S> jac = j ? jac1 : jac0;
      SP<S, int> ch = j ? chain2 : chain;
      int n;
      if (t == mjhipEQ_JOINT) {
        pv[j] = d.qpos[m.jnt_qposadr[ids[j]]];
        ref[j] = m.qpos0[m.jnt_qposadr[ids[j]]];
        n = 1;
        ch[0] = m.jnt_dofadr[ids[j]];
        jac[0] = 1;
      } else {
        pv[j] = d.ten_length[ids[j]];
        ref[j] = m.tendon_length0[ids[j]];
        const int a = d.ten_J_rowadr[ids[j]];
        n = d.ten_J_rownnz[ids[j]];
        for (int k = 0; k < n; k++) {
          ch[k] = d.ten_J_colind[a+k];
          jac[k] = d.ten_J[a+k];
        }
      }
      if (j) NV2 = n; else NV = n;
    }
    if (id1 >= 0) {
      const double dif = pv[1] - ref[1];
      cpos[0] = pv[0] - ref[0] - data[0] -
                (data[1]*dif + data[2]*dif*dif + data[3]*dif*dif*dif + data[4]*dif*dif*dif*dif);
      const double deriv = data[1] + 2*data[2]*dif + 3*data[3]*dif*dif + 4*data[4]*dif*dif*dif;
      NV = combineSparse(jac0, jac1, 1.0, -deriv, NV, NV2, chain, chain2, d.sparse_buf, bufind);
    } else {
      cpos[0] = pv[0] - ref[0] - data[0];
    }
    addRowsSparse(m, d, rc, jac0, NV, chain, cpos, (const double*)nullptr, 0.0, 1,
                  CNSTR_EQUALITY, i, status);
  }
}

template <int S, bool CONTACT = true, bool FUSED = false>
MJH_HD void makeConstraint(const mjhipModel& m, const Lane<S>& d, int* status) {
  int nv = m.nv;
  RowCount rc;
  int dsbl = m.opt.disableflags;
  // sparse mode: rows over their chains (one-entry chains of a single dof in chainbuf)
  const bool sparse = !FUSED && mjh_isSparse(&m);
  if (dsbl & mjhipDSBL_CONSTRAINT) {
    d.efc_count[0] = 0; d.efc_count[1] = 0; d.efc_count[2] = 0; d.efc_count[3] = 0;
    if (sparse) d.nJ[0] = 0;
    if constexpr (FUSED) zero(d.qfrc_constraint, nv);
    return;
  }
  // a just-added non-contact row, finished at once on the fused path
  auto added = [&](bool ok, int tp, int id, double pos, double margin, double frictionloss) {
    if constexpr (FUSED) {
      if (ok) finishNonContact(m, d, rc.nefc - 1, tp, id, pos, margin, frictionloss);
    }
  };
  SP<S> jacrow = d.jacp;       // one dense row of scratch
  SP<S, int> one = d.chainbuf;
  instantiateEquality<S, FUSED>(m, d, rc, status);
  if (!(dsbl & mjhipDSBL_FRICTIONLOSS)) {
    for (int i = 0; i < nv; i++) {
      if (m.dof_frictionloss[i] > 0) {
        if (sparse) {
          jacrow[0] = 1;
          one[0] = i;
        } else {
          zero(jacrow, nv);
          jacrow[i] = 1;
        }
        added(addConstraint1(m, d, rc, jacrow, 0, 0, m.dof_frictionloss[i], CNSTR_FRICTION_DOF,
                             i, status, 1, one), CNSTR_FRICTION_DOF, i, 0, 0,
              m.dof_frictionloss[i]);
      }
    }
    // :801-815: tendon friction on the tendon's ten_J row (dense: dropped when the row is
    // empty; sparse: when its chain is)
    for (int i = 0; i < m.ntendon; i++) {
      if (m.tendon_frictionloss[i] > 0) {
        const int ta = sparse ? d.ten_J_rowadr[i] : i*nv;
        added(addConstraint1(m, d, rc, d.ten_J + ta, 0, 0, m.tendon_frictionloss[i],
                             CNSTR_FRICTION_TENDON, i, status,
                             sparse ? d.ten_J_rownnz[i] : 0, d.ten_J_colind + (sparse ? ta : 0)),
              CNSTR_FRICTION_TENDON, i, 0, 0, m.tendon_frictionloss[i]);
      }
    }
  }
  if (!(dsbl & mjhipDSBL_LIMIT)) {
    for (int i = 0; i < m.njnt; i++) {
      if (!m.jnt_limited[i]) continue;
      double margin = m.jnt_margin[i];
      int t = m.jnt_type[i];
      if (t == mjhipJNT_SLIDE || t == mjhipJNT_HINGE) {
        double value = d.qpos[m.jnt_qposadr[i]];
        for (int side = -1; side <= 1; side += 2) {
          double dist = side * (m.jnt_range[2*i+(side+1)/2] - value);
          if (dist < margin) {
            if (sparse) {
              jacrow[0] = -(double)side;
              one[0] = m.jnt_dofadr[i];
            } else {
              zero(jacrow, nv);
              jacrow[m.jnt_dofadr[i]] = -(double)side;
            }
            added(addConstraint1(m, d, rc, jacrow, dist, margin, 0, CNSTR_LIMIT_JOINT, i, status,
                                 1, one),
                  CNSTR_LIMIT_JOINT, i, dist, margin, 0);
          }
        }
      } else if (t == mjhipJNT_BALL) {
        int adr = m.jnt_qposadr[i];
        double quat[4] = {d.qpos[adr], d.qpos[adr+1], d.qpos[adr+2], d.qpos[adr+3]};
        double angleAxis[3];
        normalize4(quat);
        quat2Vel(angleAxis, quat, 1);
        double value = normalize3(angleAxis);
        double dist = dmax(m.jnt_range[2*i], m.jnt_range[2*i+1]) - value;
        if (dist < margin) {
          if (sparse) {
            scl3(jacrow, angleAxis, -1);
            for (int k = 0; k < 3; k++) one[k] = m.jnt_dofadr[i] + k;
          } else {
            zero(jacrow, nv);
            scl3(jacrow + m.jnt_dofadr[i], angleAxis, -1);
          }
          added(addConstraint1(m, d, rc, jacrow, dist, margin, 0, CNSTR_LIMIT_JOINT, i, status,
                               3, one),
                CNSTR_LIMIT_JOINT, i, dist, margin, 0);
        }
      }
    }
    for (int i = 0; i < m.ntendon; i++) {
      if (!m.tendon_limited[i]) continue;
      double value = d.ten_length[i];
      double margin = m.tendon_margin[i];
      for (int side = -1; side <= 1; side += 2) {
        double dist = side * (m.tendon_range[2*i+(side+1)/2] - value);
        if (dist < margin) {
          if (sparse) {
            scl(jacrow, d.ten_J + d.ten_J_rowadr[i], -side, d.ten_J_rownnz[i]);
          } else {
            scl(jacrow, d.ten_J + i*nv, -side, nv);
          }
          added(addConstraint1(m, d, rc, jacrow, dist, margin, 0, CNSTR_LIMIT_TENDON, i, status,
                               sparse ? d.ten_J_rownnz[i] : 0,
                               d.ten_J_colind + (sparse ? d.ten_J_rowadr[i] : 0)),
                CNSTR_LIMIT_TENDON, i, dist, margin, 0);
        }
      }
    }
  }
  if constexpr (CONTACT) {
    if constexpr (FUSED) instantiateContactFused(m, d, rc, status);
    else instantiateContact(m, d, rc, status);
  }
  d.efc_count[0] = rc.nefc; d.efc_count[1] = rc.ne; d.efc_count[2] = rc.nf;
  d.efc_count[3] = rc.nl;
  const int nefc = rc.nefc;
  if (sparse) {                 // :2044-2104: nJ, the transpose (supernodes are AVX-only)
    d.nJ[0] = nefc ? d.efc_J_rowadr[nefc-1] + d.efc_J_rownnz[nefc-1] : 0;
    if (nefc) transposeRows(m, d, nefc);
  }
  if constexpr (FUSED) {
    constraintForce(m, d, nefc);
    return;
  }
  // mj_diagApprox :1138-1311
  for (int i = 0; i < nefc; i++) {
    int id = d.efc_id[i];
    int tp = d.efc_type[i];
    if (tp == CNSTR_EQUALITY) {
      const int size = m.eq_type[id] == mjhipEQ_CONNECT ? 3 : (m.eq_type[id] == mjhipEQ_WELD ? 6 : 1);
      for (int k = 0; k < size; k++) d.efc_diagApprox[i+k] = eqDiagApprox(m, id, k);
      i += size - 1;
    } else if (tp == CNSTR_FRICTION_DOF) {
      d.efc_diagApprox[i] = m.dof_invweight0[id];
    } else if (tp == CNSTR_LIMIT_JOINT) {
      d.efc_diagApprox[i] = m.dof_invweight0[m.jnt_dofadr[id]];
    } else if (tp == CNSTR_LIMIT_TENDON || tp == CNSTR_FRICTION_TENDON) {
      d.efc_diagApprox[i] = m.tendon_invweight0[id];
    } else if constexpr (CONTACT) {   // contact rows
      int dim = d.con_dim[id];
      double tran = 0, rot = 0;
      for (int side = 0; side < 2; side++) {
        int b = m.geom_bodyid[d.con_geom[2*id+side]];
        tran += m.body_invweight0[2*b] * 1.0;
        rot += m.body_invweight0[2*b+1] * 1.0;
      }
      if (tp == CNSTR_CONTACT_FRICTIONLESS) {
        d.efc_diagApprox[i] = tran;
      } else if (tp == CNSTR_CONTACT_ELLIPTIC) {
        for (int j = 0; j < dim; j++) d.efc_diagApprox[i+j] = j < 3 ? tran : rot;
        i += dim - 1;
      } else {
        for (int j = 0; j < dim-1; j++) {
          double fri = d.con_friction[5*id+j];
          double v = tran + fri*fri*(j < 2 ? tran : rot);
          d.efc_diagApprox[i+2*j] = v;
          d.efc_diagApprox[i+2*j+1] = v;
        }
        i += 2*dim - 3;
      }
    }
  }
  // mj_makeImpedance :1494-1608; a pyramidal contact's 2*(condim-1) rows share one impedance
  for (int i = 0; i < nefc; i++) {
    int id = d.efc_id[i];
    int tp = d.efc_type[i];
    double solref[2], solimp[5], solreffriction[2] = {0, 0};
    const bool iscontact = CONTACT && (tp == CNSTR_CONTACT_FRICTIONLESS ||
                                       tp == CNSTR_CONTACT_PYRAMIDAL ||
                                       tp == CNSTR_CONTACT_ELLIPTIC);
    if (iscontact) {
      for (int k = 0; k < 2; k++) solref[k] = d.con_solref[2*id+k];
      for (int k = 0; k < 5; k++) solimp[k] = d.con_solimp[5*id+k];
      for (int k = 0; k < 2; k++) solreffriction[k] = d.con_solreffriction[2*id+k];
    } else {
      rowSolParam(m, tp, id, solref, solimp);
    }
    int dim = (CONTACT && tp == CNSTR_CONTACT_PYRAMIDAL) ? 2*(d.con_dim[id]-1) :
              ((CONTACT && tp == CNSTR_CONTACT_ELLIPTIC) ? d.con_dim[id] : 1);
    double ipos = d.efc_pos[i];
    if (tp == CNSTR_EQUALITY && (m.eq_type[id] == mjhipEQ_CONNECT || m.eq_type[id] == mjhipEQ_WELD)) {
      dim = m.eq_type[id] == mjhipEQ_WELD ? 6 : 3;      // getposdim :1392-1422
      ipos = sqrt(dot(d.efc_pos + i, d.efc_pos + i, dim));
    }
    double kb[4];
    rowImpedance(m, tp, solref, solimp, ipos, d.efc_margin[i], kb);
    // elliptic friction rows: K = 0, B from solreffriction when set (:1511-1524; its
    // getsolparam clamps :1358-1366)
    double kbf[4] = {0, kb[1], kb[2], kb[3]};
    if (CONTACT && tp == CNSTR_CONTACT_ELLIPTIC) {
      double sf[2] = {solreffriction[0], solreffriction[1]};
      if ((sf[0] > 0) ^ (sf[1] > 0)) { sf[0] = 0; sf[1] = 0; }
      if (!(m.opt.disableflags & mjhipDSBL_REFSAFE) && sf[0] > 0) {
        sf[0] = dmax(sf[0], 2*m.opt.timestep);
      }
      const double* ref = (sf[0] || sf[1]) ? sf : solref;
      const double dmaxi = dmin(mjhipMAXIMP, dmax(mjhipMINIMP, solimp[1]));
      kbf[1] = ref[1] > 0 ? 2 / dmax(MINVAL, dmaxi*ref[0]) : -ref[1] / dmax(MINVAL, dmaxi);
    }
    for (int j = 0; j < dim; j++) {
      int r = i + j;
      d.efc_R[r] = dmax(MINVAL, (1-kb[2])*d.efc_diagApprox[r]/kb[2]);
      const double* k4 = (CONTACT && tp == CNSTR_CONTACT_ELLIPTIC && j > 0) ? kbf : kb;
      for (int k = 0; k < 4; k++) d.efc_KBIP[4*r+k] = k4[k];
    }
    i += dim - 1;
  }
  // frictional contacts: R in the friction directions, contact mu (:1562-1598)
  for (int i = rc.nf; CONTACT && i < nefc; i++) {
    if (d.efc_type[i] == CNSTR_CONTACT_ELLIPTIC) {
      int id = d.efc_id[i], dim = d.con_dim[id];
      d.efc_R[i+1] = d.efc_R[i]/dmax(MINVAL, m.opt.impratio);
      const double f0 = d.con_friction[5*id];
      d.con_mu[id] = f0 * sqrt(d.efc_R[i+1]/d.efc_R[i]);
      for (int j = 1; j < dim-1; j++) {
        const double fj = d.con_friction[5*id+j];
        d.efc_R[i+j+1] = d.efc_R[i+1]*f0*f0/(fj*fj);
      }
      i += dim - 1;
    } else if (d.efc_type[i] == CNSTR_CONTACT_PYRAMIDAL) {
      int id = d.efc_id[i], dim = d.con_dim[id];
      d.efc_R[i+1] = d.efc_R[i]/dmax(MINVAL, m.opt.impratio);
      double mu = d.con_friction[5*id] * sqrt(d.efc_R[i+1]/d.efc_R[i]);
      d.con_mu[id] = mu;
      double Rpy = 2*mu*mu*d.efc_R[i];
      for (int j = 0; j < 2*(dim-1); j++) d.efc_R[i+j] = Rpy;
      i += 2*(dim-1) - 1;
    }
  }
  for (int i = 0; i < nefc; i++) d.efc_D[i] = 1 / d.efc_R[i];
  for (int i = 0; i < nefc; i++) {
    d.efc_diagApprox[i] = d.efc_R[i] * d.efc_KBIP[4*i+2] / (1-d.efc_KBIP[4*i+2]);
  }
}

// mj_referenceConstraint :2362-2375 (efc_vel = mj_mulJacVec, dense or sparse)
// The row loops here and in invConstraint run eight rows at a time: a chunk's loads are
// issued before its stores, so it waits once for the stores before it, not once per row
// (the device orders a load after every older store it cannot prove disjoint). Same
// operations per row.
constexpr int kRowChunk = 8;

template <int S>
MJH_HD void referenceConstraint(const mjhipModel& m, const Lane<S>& d) {
  int nefc = d.efc_count[0];
  const bool sparse = mjh_isSparse(&m);
  for (int i0 = 0; i0 < nefc; i0 += kRowChunk) {
    double vel[kRowChunk], aref[kRowChunk];
#pragma unroll
    for (int u = 0; u < kRowChunk; u++) {
      const int i = i0 + u;
      if (i >= nefc) continue;
      vel[u] = sparse ? jacRowDot(d, i, d.qvel) : dot(d.efc_J + i*m.nv, d.qvel, m.nv);
      aref[u] = -d.efc_KBIP[4*i+1]*vel[u]
                -d.efc_KBIP[4*i]*d.efc_KBIP[4*i+2]*(d.efc_pos[i]-d.efc_margin[i]);
    }
#pragma unroll
    for (int u = 0; u < kRowChunk; u++) {
      if (i0 + u >= nefc) continue;
      d.efc_vel[i0 + u] = vel[u];
      d.efc_aref[i0 + u] = aref[u];
    }
  }
}

// mj_invConstraint engine_inverse.c:169-192 with mj_constraintUpdate_island :2387-2549
// (island < 0, no cost; elliptic-cone rows come only from contacts: outside this subset)
template <int S>
MJH_HD void invConstraint(const mjhipModel& m, const Lane<S>& d) {
  int nv = m.nv, nefc = d.efc_count[0];
  if (!nefc) {
    zero(d.qfrc_constraint, nv);
    return;
  }
  int ne = d.efc_count[1], nf = d.efc_count[2];
  const bool sparse = mjh_isSparse(&m);
  for (int i0 = 0; i0 < nefc; i0 += kRowChunk) {
    double jar[kRowChunk];
#pragma unroll
    for (int u = 0; u < kRowChunk; u++) {
      const int i = i0 + u;
      if (i >= nefc) continue;
      jar[u] = (sparse ? jacRowDot(d, i, d.qacc) : dot(d.efc_J + i*nv, d.qacc, nv)) -
               d.efc_aref[i];
    }
#pragma unroll
    for (int u = 0; u < kRowChunk; u++) {
      const int i = i0 + u;
      if (i >= nefc) continue;
      d.jar[i] = jar[u];
      d.efc_force[i] = -d.efc_D[i] * jar[u];
    }
  }
  for (int i = 0; i < nefc; i++) {
    double jr = d.jar[i];
    if (i < ne) {
      d.efc_state[i] = CNSTRSTATE_QUADRATIC;
    } else if (i < ne + nf) {
      double Rf = d.efc_R[i] * d.efc_frictionloss[i];
      if (jr <= -Rf) {
        d.efc_force[i] = d.efc_frictionloss[i];
        d.efc_state[i] = CNSTRSTATE_LINEARNEG;
      } else if (jr >= Rf) {
        d.efc_force[i] = -d.efc_frictionloss[i];
        d.efc_state[i] = CNSTRSTATE_LINEARPOS;
      } else {
        d.efc_state[i] = CNSTRSTATE_QUADRATIC;
      }
    } else if (d.efc_type[i] != CNSTR_CONTACT_ELLIPTIC) {
      if (jr >= 0) {
        d.efc_force[i] = 0;
        d.efc_state[i] = CNSTRSTATE_SATISFIED;
      } else {
        d.efc_state[i] = CNSTRSTATE_QUADRATIC;
      }
    } else {
      // elliptic cone :2459-2540 (no cost, no cone Hessian)
      const int id = d.efc_id[i], dim = d.con_dim[id];
      const double mu = d.con_mu[id];
      double U[6];
      U[0] = jr*mu;
      for (int j = 1; j < dim; j++) U[j] = d.jar[i+j]*d.con_friction[5*id+j-1];
      const double N = U[0];
      const double T = sqrt(dot(U + 1, U + 1, dim - 1));
      int state;
      if (N >= mu*T || (T <= 0 && N >= 0)) {
        for (int j = 0; j < dim; j++) d.efc_force[i+j] = 0;
        state = CNSTRSTATE_SATISFIED;
      } else if (mu*N + T <= 0 || (T <= 0 && N < 0)) {
        state = CNSTRSTATE_QUADRATIC;
      } else {
        const double Dm = d.efc_D[i] / (mu*mu*(1 + mu*mu));
        const double NmT = N - mu*T;
        const double f0 = -Dm*NmT*mu;
        d.efc_force[i] = f0;
        for (int j = 1; j < dim; j++) d.efc_force[i+j] = -f0/T*U[j]*d.con_friction[5*id+j-1];
        state = CNSTRSTATE_CONE;
      }
      for (int j = 0; j < dim; j++) d.efc_state[i+j] = state;
      i += dim - 1;
    }
  }
  if (sparse) {                         // mju_mulMatVecSparse over the rows of efc_JT
    for (int j0 = 0; j0 < nv; j0 += kRowChunk) {
      double q[kRowChunk];
#pragma unroll
      for (int u = 0; u < kRowChunk; u++) {
        if (j0 + u < nv) q[u] = jacColDot(d, j0 + u, d.efc_force);
      }
#pragma unroll
      for (int u = 0; u < kRowChunk; u++) {
        if (j0 + u < nv) d.qfrc_constraint[j0 + u] = q[u];
      }
    }
  } else {
    mulMatTVec(d.qfrc_constraint, d.efc_J, d.efc_force, nefc, nv);
  }
}

//---------------------------------- engine_inverse.c -----------------------------------------

// mj_invPosition :37-68 (mj_flex: no flexes)
template <int S, bool CONTACT = true, bool FUSED = false>
MJH_HD void invPosition(const mjhipModel& m, const Lane<S>& d, int* status) {
  kinematics(m, d);
  MJH_PHASE(1);
  comPos(m, d);
  camlight(m, d);
  tendon(m, d);
  MJH_PHASE(2);
  crb(m, d);
  factorM(m, d, status);
  MJH_PHASE(3);
  if constexpr (CONTACT) collision(m, d, status);
  else d.con_count[0] = 0;
  MJH_PHASE(4);
  makeConstraint<S, CONTACT, FUSED>(m, d, status);
  MJH_PHASE(5);
  transmission(m, d);
}

// mj_invVelocity :73-76 -> mj_fwdVelocity engine_forward.c:193-231
template <int S, bool FUSED = false>
MJH_HD void invVelocity(const mjhipModel& m, const Lane<S>& d) {
  int nv = m.nv;
  if (mjh_isSparse(&m)) {                  // engine_forward.c:206-212, sparse
    for (int r = 0; r < m.ntendon; r++) {
      const int a = d.ten_J_rowadr[r];
      d.ten_velocity[r] = dotSparse(d.ten_J + a, d.qvel, d.ten_J_rownnz[r], d.ten_J_colind + a);
    }
  } else {
    for (int r = 0; r < m.ntendon; r++) d.ten_velocity[r] = dot(d.ten_J + r*nv, d.qvel, nv);
  }
  if (!(m.opt.disableflags & mjhipDSBL_ACTUATION)) {
    for (int r = 0; r < m.nu; r++) {
      int adr = m.moment_rowadr[r];
      d.actuator_velocity[r] = dotSparse(d.actuator_moment + adr, d.qvel, m.moment_rownnz[r],
                                         m.moment_colind + adr);
    }
  }
  comVel(m, d);
  passive(m, d);
  if constexpr (!FUSED) referenceConstraint(m, d);   // fused: done with the rows
  rne(m, d, 0, d.qfrc_bias);
}

// mj_inverseSkip :197-261 (sensors/energy: none in this subset)
// mj_solveLD :1629-1707 on the qLD factor (one right-hand side), in place
template <int S>
MJH_HD void solveM(const mjhipModel& m, const Lane<S>& d, SP<S> x) {
  const int nv = m.nv;
  for (int i = nv-1; i > 0; i--) {
    if (m.dof_simplenum[i]) continue;
    int start = m.C_rowadr[i], end = start + m.C_rownnz[i] - 1;
    double x_i = x[i];
    if (x_i) {
      for (int adr = start; adr < end; adr++) x[m.C_colind[adr]] -= d.qLD[adr] * x_i;
    }
  }
  for (int i = 0; i < nv; i++) x[i] *= d.qLDiagInv[i];
  for (int i = 1; i < nv; i++) {
    if (m.dof_simplenum[i]) {
      i += m.dof_simplenum[i] - 1;
      continue;
    }
    int dd = m.C_rownnz[i] - 1;
    if (dd > 0) {
      int adr = m.C_rowadr[i];
      x[i] -= dotSparse(d.qLD + adr, x, dd, m.C_colind + adr);
    }
  }
}

// mj_mulM engine_support.c:966-1017
template <int S>
MJH_HD void mulM(const mjhipModel& m, const Lane<S>& d, SP<S> res, SP<S> vec) {
  const int nv = m.nv;
  zero(res, nv);
  for (int i = 0; i < nv; i++) {
    int adr = m.dof_Madr[i];
    res[i] = d.qM[adr]*vec[i];
    if (m.dof_simplenum[i]) continue;
    int j = m.dof_parentid[i];
    while (j >= 0) {
      adr++;
      res[i] += d.qM[adr]*vec[j];
      res[j] += d.qM[adr]*vec[i];
      j = m.dof_parentid[j];
    }
  }
}

// dense value of the sparse actuator_moment row `i` at column `col`
template <int S>
MJH_HD double momentAt(const mjhipModel& m, const Lane<S>& d, int i, int col) {
  int adr = m.moment_rowadr[i];
  for (int k = 0; k < m.moment_rownnz[i]; k++) {
    if (m.moment_colind[adr+k] == col) return d.actuator_moment[adr+k];
  }
  return 0;
}

// ten_J of tendon t at dof col: the dense row, or the compressed row of a sparse-mode model
template <int S>
MJH_HD double tenJAt(const mjhipModel& m, const Lane<S>& d, int t, int col) {
  if (!mjh_isSparse(&m)) return d.ten_J[t*m.nv + col];
  const int a = d.ten_J_rowadr[t], n = d.ten_J_rownnz[t];
  for (int k = 0; k < n; k++) {
    if (d.ten_J_colind[a+k] == col) return d.ten_J[a+k];
  }
  return 0;
}

// qDeriv(r, c) of mjd_smooth_vel(flg_bias = 0) (engine_derivative.c:1522-1536): actuator
// velocity terms (mjd_actuator_vel :812-870, addJTBJ :693-724), then dof and tendon damping
// (mjd_passive_vel :1432-1519), in the reference's order of accumulation
template <int S>
MJH_HD double qDerivAt(const mjhipModel& m, const Lane<S>& d, int r, int c) {
  double q = 0;
  if (!(m.opt.disableflags & mjhipDSBL_ACTUATION)) {
    for (int i = 0; i < m.nu; i++) {
      double bias_vel = 0, gain_vel = 0;
      if (m.actuator_biastype[i] == mjhipBIAS_AFFINE) bias_vel = m.actuator_biasprm[10*i+2];
      if (m.actuator_gaintype[i] == mjhipGAIN_AFFINE) gain_vel = m.actuator_gainprm[10*i+2];
      if (gain_vel != 0) bias_vel += gain_vel * d.ctrl[i];
      if (bias_vel != 0) {
        double mr = momentAt(m, d, i, r);
        if (mr) q += momentAt(m, d, i, c) * (mr * bias_vel);
      }
    }
  }
  if (!(m.opt.disableflags & mjhipDSBL_PASSIVE)) {
    if (r == c) q -= m.dof_damping[r];
    for (int t = 0; t < m.ntendon; t++) {
      if (m.tendon_damping[t] > 0) {
        // addJTBJ :693-724, or addJTBJSparse :729-755 for a sparse-mode model, whose only
        // extra terms are exact zeros (structural entries of value 0)
        double B = -m.tendon_damping[t];
        const double Jr = tenJAt(m, d, t, r);
        if (Jr) q += tenJAt(m, d, t, c) * (Jr * B);
      }
    }
  }
  return q;
}

//---------------------------------- engine_derivative.c (implicit integrator) ----------------

// 6x6 Jacobians of the spatial helpers (engine_derivative.c:65-213), row-major, zero
// elsewhere: crossMotion(vel, v) and crossForce(vel, f) in vel, crossForce in f,
// mulInertVec in v
MJH_HD void set36(double D[36], const int (*rc)[2], const double* val, int n) {
  for (int k = 0; k < 36; k++) D[k] = 0;
  for (int k = 0; k < n; k++) D[rc[k][0]*6 + rc[k][1]] = val[k];
}
MJH_HD void crossMotionVel(double D[36], const double v[6]) {
  const int rc[18][2] = {{0,2}, {0,1}, {1,2}, {1,0}, {2,1}, {2,0}, {3,2}, {3,1}, {3,5}, {3,4},
                         {4,2}, {4,0}, {4,5}, {4,3}, {5,1}, {5,0}, {5,4}, {5,3}};
  const double val[18] = {-v[1], v[2], v[0], -v[2], -v[0], v[1], -v[4], v[5], -v[1], v[2],
                          v[3], -v[5], v[0], -v[2], -v[3], v[4], -v[0], v[1]};
  set36(D, rc, val, 18);
}
MJH_HD void crossForceVel(double D[36], const double f[6]) {
  const int rc[18][2] = {{0,2}, {0,1}, {0,5}, {0,4}, {1,2}, {1,0}, {1,5}, {1,3}, {2,1}, {2,0},
                         {2,4}, {2,3}, {3,2}, {3,1}, {4,2}, {4,0}, {5,1}, {5,0}};
  const double val[18] = {-f[1], f[2], -f[4], f[5], f[0], -f[2], f[3], -f[5], -f[0], f[1],
                          -f[3], f[4], -f[4], f[5], f[3], -f[5], -f[3], f[4]};
  set36(D, rc, val, 18);
}
MJH_HD void crossForceFrc(double D[36], const double v[6]) {
  const int rc[18][2] = {{0,1}, {0,2}, {0,4}, {0,5}, {1,0}, {1,2}, {1,3}, {1,5}, {2,0}, {2,1},
                         {2,3}, {2,4}, {3,4}, {3,5}, {4,3}, {4,5}, {5,3}, {5,4}};
  const double val[18] = {-v[2], v[1], -v[5], v[4], v[2], -v[0], v[5], -v[3], -v[1], v[0],
                          -v[4], v[3], -v[2], v[1], v[2], -v[0], -v[1], v[0]};
  set36(D, rc, val, 18);
}
MJH_HD void mulInertVecVel(double D[36], const double i[10]) {
  const int rc[24][2] = {{0,0}, {0,1}, {0,2}, {0,4}, {0,5}, {1,0}, {1,1}, {1,2}, {1,3}, {1,5},
                         {2,0}, {2,1}, {2,2}, {2,3}, {2,4}, {3,1}, {3,2}, {3,3}, {4,2}, {4,0},
                         {4,4}, {5,0}, {5,1}, {5,5}};
  const double val[24] = {i[0], i[3], i[4], -i[8], i[7], i[3], i[1], i[5], i[8], -i[6],
                          i[4], i[5], i[2], -i[7], i[6], i[8], -i[7], i[9], i[6], -i[8],
                          i[9], i[7], -i[6], i[9]};
  set36(D, rc, val, 24);
}
MJH_HD void transpose6(double r[36], const double a[36]) {
  for (int i = 0; i < 6; i++) for (int j = 0; j < 6; j++) r[j*6+i] = a[i*6+j];
}

// res (r1 x 6) = a (r1 x 6) * b (6 x 6), mju_mulMatMat engine_util_blas.c:818-832 (zero
// entries of `a` skipped)
template <class R, class A> MJH_HD void mulMat6(R res, A a, const double* b, int r1) {
  for (int i = 0; i < r1; i++) {
    double out[6] = {0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 6; k++) {
      double t = a[6*i+k];
      if (t) for (int c = 0; c < 6; c++) out[c] += b[6*k+c]*t;
    }
    for (int c = 0; c < 6; c++) res[6*i+c] = out[c];
  }
}

// number of dof ancestors of dof j (engine_derivative.c:542)
MJH_HD int dofJadr(const mjhipModel& m, int j) {
  return (j < m.nv - 1 ? m.dof_Madr[j+1] : m.nM) - (m.dof_Madr[j] + 1);
}

// copyFromParent :484-500 (body n's B row begins with its ancestors' dofs, as the parent's)
template <int S> MJH_HD void bCopyFromParent(const mjhipModel& m, SP<S> mat, int n) {
  if (n == 0 || m.body_weldid[m.body_parentid[n]] == 0) return;
  int ndof = 0;
  for (int p = m.body_weldid[m.body_parentid[n]]; p > 0; p = m.body_weldid[m.body_parentid[p]]) {
    ndof += m.body_dofnum[p];
  }
  copy(mat + 6*m.B_rowadr[n], mat + 6*m.B_rowadr[m.body_parentid[n]], 6*ndof);
}

// addToParent :505-531 (child columns are a subset of the parent's)
template <int S> MJH_HD void bAddToParent(const mjhipModel& m, SP<S> mat, int n) {
  if (n == 0 || m.body_weldid[m.body_parentid[n]] == 0) return;
  const int np = m.body_parentid[n];
  const int* cn = m.B_colind + m.B_rowadr[n];
  const int* cp = m.B_colind + m.B_rowadr[np];
  for (int i = 0, ip = 0; i < m.B_rownnz[n] && ip < m.B_rownnz[np]; ip++) {
    if (cn[i] == cp[ip]) {
      addTo(mat + 6*(m.B_rowadr[np] + ip), mat + 6*(m.B_rowadr[n] + i), 6);
      i++;
    }
  }
}

// mjd_comVel_vel :535-600: Dcvel (B sparsity) and Dcdofdot (D sparsity), 6 per nonzero
template <int S> MJH_HD void comVelVel(const mjhipModel& m, const Lane<S>& d) {
  double mat[36], matT[36], cd[6];
  for (int i = 1; i < m.nbody; i++) {
    bCopyFromParent(m, d.Dcvel, i);
    SP<S> row = d.Dcvel + 6*m.B_rowadr[i];
    const int last = m.body_dofadr[i] + m.body_dofnum[i];
    for (int j = m.body_dofadr[i]; j < last; j++) {
      int Jadr = dofJadr(m, j);
      const int t = m.jnt_type[m.dof_jntid[j]];
      int nrot = 1;
      if (t == mjhipJNT_FREE) {           // translations: Dcdofdot stays zero
        for (int k = 0; k < 3; k++) addTo(row + 6*(Jadr + k), d.cdof + 6*(j + k), 6);
        j += 3;
        Jadr += 3;
        nrot = 3;
      } else if (t == mjhipJNT_BALL) {
        nrot = 3;
      }
      for (int k = 0; k < nrot; k++) {
        for (int c = 0; c < 6; c++) cd[c] = d.cdof[6*(j + k) + c];
        crossMotionVel(mat, cd);
        transpose6(matT, mat);
        mulMat6(d.Dcdofdot + 6*m.D_rowadr[j + k], row, matT, Jadr + k);
      }
      for (int k = 0; k < nrot; k++) addTo(row + 6*(Jadr + k), d.cdof + 6*(j + k), 6);
      j += nrot - 1;
    }
  }
}

// mjd_rne_vel :604-690: qDeriv -= d qfrc_bias / d qvel on the D sparsity
template <int S> MJH_HD void rneVel(const mjhipModel& m, const Lane<S>& d) {
  zero(d.Dcvel, 6*m.nB);
  zero(d.Dcacc, 6*m.nB);
  zero(d.Dcfrc, 6*m.nB);
  zero(d.Dcdofdot, 6*m.nD);
  comVelVel(m, d);
  double mat[36], mat1[36], mat2[36], dmul[36], tmp[6], in[10], vel[6];
  for (int i = 1; i < m.nbody; i++) {
    bCopyFromParent(m, d.Dcacc, i);
    const int nnz = m.B_rownnz[i];
    SP<S> acc = d.Dcacc + 6*m.B_rowadr[i];
    const int last = m.body_dofadr[i] + m.body_dofnum[i];
    for (int j = m.body_dofadr[i]; j < last; j++) {
      addTo(acc + 6*dofJadr(m, j), d.cdof_dot + 6*j, 6);
      addToScl(acc, d.Dcdofdot + 6*m.D_rowadr[j], d.qvel[j], 6*nnz);
    }
    for (int k = 0; k < 10; k++) in[k] = d.cinert[10*i+k];
    for (int k = 0; k < 6; k++) vel[k] = d.cvel[6*i+k];
    mulInertVecVel(dmul, in);
    transpose6(mat1, dmul);
    mulMat6(d.Dcfrc + 6*m.B_rowadr[i], acc, mat1, nnz);
    mulInertVec(tmp, in, vel);
    crossForceVel(mat, tmp);
    crossForceFrc(mat1, vel);
    for (int r = 0; r < 6; r++) {         // mat2 = mat1 * dmul (mju_mulMatMat)
      double out[6] = {0, 0, 0, 0, 0, 0};
      for (int k = 0; k < 6; k++) {
        double t = mat1[6*r+k];
        if (t) for (int c = 0; c < 6; c++) out[c] += dmul[6*k+c]*t;
      }
      for (int c = 0; c < 6; c++) mat2[6*r+c] = out[c];
    }
    for (int k = 0; k < 36; k++) mat[k] += mat2[k];
    transpose6(mat1, mat);
    mulMat6(d.Dtmp, d.Dcvel + 6*m.B_rowadr[i], mat1, nnz);
    addTo(d.Dcfrc + 6*m.B_rowadr[i], d.Dtmp, 6*nnz);
  }
  for (int i = m.nbody - 1; i > 0; i--) bAddToParent(m, d.Dcfrc, i);
  for (int j = 0; j < m.nv; j++) {
    const int i = m.dof_bodyid[j], nnz = m.B_rownnz[i];
    SP<S> fr = d.Dcfrc + 6*m.B_rowadr[i];
    SP<S> q = d.qDeriv + m.D_rowadr[j];
    for (int k = 0; k < nnz; k++) q[k] -= dot6(fr + 6*k, d.cdof + 6*j);
  }
}

//---------------------------------- engine_derivative.c (fluid) ------------------------------

// addJTBJ :693-724: qDeriv (D sparsity) += J' B J for the n x n B and the n rows of J (Dtmp)
template <int S>
MJH_HD void addJTBJ(const mjhipModel& m, const Lane<S>& d, SP<S> J, const double* B, int n) {
  const int nv = m.nv;
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < n; j++) {
      if (!B[i*n+j]) continue;
      for (int k = 0; k < nv; k++) {
        const double jik = J[i*nv+k];
        if (!jik) continue;
        const double s = jik * B[i*n+j];
        const int adr = m.D_rowadr[k], end = adr + m.D_rownnz[k];
        for (int a = adr; a < end; a++) d.qDeriv[a] += J[j*nv + m.D_colind[a]] * s;
      }
    }
  }
}

// :898-909 addToQuadrant (the reference indexes B column-major in 3x3 blocks)
MJH_HD void addToQuadrant(double* B, const double D[9], int col_quad, int row_quad) {
  const int r = 3*row_quad, c = 3*col_quad;
  for (int k = 0; k < 3; k++) {
    for (int l = 0; l < 3; l++) B[6*(c+k) + r+l] += D[3*k+l];
  }
}

// :38-61 mjd_cross
MJH_HD void dcross(const double a[3], const double b[3], double* Da, double* Db) {
  for (int k = 0; k < 9; k++) Da[k] = Db[k] = 0;
  Da[1] =  b[2]; Da[2] = -b[1]; Da[3] = -b[2]; Da[5] =  b[0]; Da[6] =  b[1]; Da[7] = -b[0];
  Db[1] = -a[2]; Db[2] =  a[1]; Db[3] =  a[2]; Db[5] = -a[0]; Db[6] = -a[1]; Db[7] =  a[0];
}

// the ellipsoid model's 6x6 B of one geom (:1239-1259): Magnus, Kutta, viscous drag and
// torque (:962-1161) and added mass (:916-957) in the reference's order of accumulation
MJH_HD void ellipsoidFluidB(double* B, const double lv[6], double rho, double mu,
                            const double s[3], const double* c, bool symmetric) {
  auto mx = [](double a, double b) { return a > b ? a : b; };
  auto mn = [](double a, double b) { return a < b ? a : b; };
  double D[9], Da[9], Db[9];
  for (int k = 0; k < 36; k++) B[k] = 0;
  const double blunt = c[1], slender = c[2], angdrag = c[3], kutta = c[4], magnus = c[5];
  const double* vm = c + 6;
  const double* vi = c + 9;
  {                                       // mjd_magnus_force
    const double volume = 4.0/3.0 * mjhipPI * s[0] * s[1] * s[2];
    const double coef = magnus * rho * volume;
    const double lin[3] = {coef * lv[3], coef * lv[4], coef * lv[5]};
    const double ang[3] = {coef * lv[0], coef * lv[1], coef * lv[2]};
    dcross(ang, lin, Da, Db);
    addToQuadrant(B, Da, 1, 0);
    addToQuadrant(B, Db, 1, 1);
  }
  const double a = (s[1]*s[2])*(s[1]*s[2]), b = (s[2]*s[0])*(s[2]*s[0]);
  const double cz = (s[0]*s[1])*(s[0]*s[1]);
  const double aa = a*a, bb = b*b, cc = cz*cz;
  const double x = lv[3], y = lv[4], z = lv[5];
  const double xx = x*x, yy = y*y, zz = z*z, xy = x*y, yz = y*z, xz = x*z;
  const double pden = aa*xx + bb*yy + cc*zz;
  const double pnum = a*xx + b*yy + cz*zz;
  {                                       // mjd_kutta_lift
    const double norm2 = xx + yy + zz;
    const double df_denom = mjhipPI * kutta * rho / mx(MINVAL, sqrt(pden * pnum * norm2));
    const double dfx = yy * (a - b) + zz * (a - cz);
    const double dfy = xx * (b - a) + zz * (b - cz);
    const double dfz = xx * (cz - a) + yy * (cz - b);
    const double proj_term = pnum / mx(MINVAL, pden);
    const double cos_term = pnum / mx(MINVAL, norm2);
    D[0] = a-a;  D[1] = b-a;  D[2] = cz-a;
    D[3] = a-b;  D[4] = b-b;  D[5] = cz-b;
    D[6] = a-cz; D[7] = b-cz; D[8] = cz-cz;
    for (int k = 0; k < 9; k++) D[k] = D[k]*(2 * pnum);
    const double inner[3] = {aa * proj_term - a + cos_term, bb * proj_term - b + cos_term,
                             cc * proj_term - cz + cos_term};
    addToScl3(D + 0, inner, dfx);
    addToScl3(D + 3, inner, dfy);
    addToScl3(D + 6, inner, dfz);
    D[0] *= xx; D[1] *= xy; D[2] *= xz;
    D[3] *= xy; D[4] *= yy; D[5] *= yz;
    D[6] *= xz; D[7] *= yz; D[8] *= zz;
    D[0] -= dfx * pnum;
    D[4] -= dfy * pnum;
    D[8] -= dfz * pnum;
    for (int k = 0; k < 9; k++) D[k] = D[k]*df_denom;
    addToQuadrant(B, D, 1, 1);
  }
  const double dmax = mx(mx(s[0], s[1]), s[2]);
  const double dmin = mn(mn(s[0], s[1]), s[2]);
  const double dmid = s[0] + s[1] + s[2] - dmax - dmin;
  const double eqD = 2.0/3.0 * (s[0] + s[1] + s[2]);
  {                                       // mjd_viscous_drag
    const double Amax = mjhipPI * dmax * dmid;
    const double dA = mjhipPI / mx(MINVAL, sqrt(pnum*pnum*pnum * pden));
    const double Aproj = mjhipPI * sqrt(pden/mx(MINVAL, pnum));
    const double norm = sqrt(xx + yy + zz);
    const double inv_norm = 1.0 / mx(MINVAL, norm);
    const double lin_coef = mu * 3.0 * mjhipPI * eqD;
    const double quad_coef = rho * (Aproj*blunt + slender*(Amax - Aproj));
    const double Ac = rho * norm * (blunt - slender);
    const double dAv[3] = {Ac * dA * a * x * (b * yy * (a - b) + cz * zz * (a - cz)),
                           Ac * dA * b * y * (a * xx * (b - a) + cz * zz * (b - cz)),
                           Ac * dA * cz * z * (a * xx * (cz - a) + b * yy * (cz - b))};
    D[0] = xx; D[1] = xy; D[2] = xz;
    D[3] = xy; D[4] = yy; D[5] = yz;
    D[6] = xz; D[7] = yz; D[8] = zz;
    const double inner = xx + yy + zz;
    D[0] += inner; D[4] += inner; D[8] += inner;
    const double sc = -quad_coef*inv_norm;
    for (int k = 0; k < 9; k++) D[k] = D[k]*sc;
    addToScl3(D + 0, dAv, -x);
    addToScl3(D + 3, dAv, -y);
    addToScl3(D + 6, dAv, -z);
    D[0] -= lin_coef; D[4] -= lin_coef; D[8] -= lin_coef;
    addToQuadrant(B, D, 1, 1);
  }
  {                                       // mjd_viscous_torque
    const double lin_visc = mjhipPI * eqD*eqD*eqD;
    const double Imax = 8.0/15.0 * mjhipPI * dmid * (dmax*dmax)*(dmax*dmax);
    double II[3];
    for (int k = 0; k < 3; k++) {         // ellipsoid_max_moment (:887-892)
      II[k] = 8.0/15.0 * mjhipPI * s[k] * pow4(mx(s[(k+1) % 3], s[(k+2) % 3]));
    }
    const double ax = lv[0], ay = lv[1], az = lv[2];
    const double mc[3] = {angdrag*II[0] + slender*(Imax - II[0]),
                          angdrag*II[1] + slender*(Imax - II[1]),
                          angdrag*II[2] + slender*(Imax - II[2])};
    const double mv[3] = {ax * mc[0], ay * mc[1], az * mc[2]};
    const double density = rho / mx(MINVAL, sqrt(mv[0]*mv[0] + mv[1]*mv[1] + mv[2]*mv[2]));
    const double msq[3] = {-density * ax * mc[0] * mc[0], -density * ay * mc[1] * mc[1],
                           -density * az * mc[2] * mc[2]};
    const double lin_coef = mu * lin_visc;
    for (int k = 0; k < 9; k++) D[k] = 0;
    D[0] = D[4] = D[8] = ax*msq[0] + ay*msq[1] + az*msq[2] - lin_coef;
    addToScl3(D, msq, ax);
    addToScl3(D + 3, msq, ay);
    addToScl3(D + 6, msq, az);
    addToQuadrant(B, D, 0, 0);
  }
  {                                       // mjd_addedMassForces
    const double lin[3] = {lv[3], lv[4], lv[5]}, ang[3] = {lv[0], lv[1], lv[2]};
    const double plin[3] = {rho*vm[0]*lin[0], rho*vm[1]*lin[1], rho*vm[2]*lin[2]};
    const double pang[3] = {rho*vi[0]*ang[0], rho*vi[1]*ang[1], rho*vi[2]*ang[2]};
    dcross(pang, ang, Da, Db);
    addToQuadrant(B, Db, 0, 0);
    for (int k = 0; k < 9; k++) Da[k] *= rho * vi[k % 3];
    addToQuadrant(B, Da, 0, 0);
    dcross(plin, lin, Da, Db);
    addToQuadrant(B, Db, 0, 1);
    for (int k = 0; k < 9; k++) Da[k] *= rho * vm[k % 3];
    addToQuadrant(B, Da, 0, 1);
    dcross(plin, ang, Da, Db);
    addToQuadrant(B, Db, 1, 0);
    for (int k = 0; k < 9; k++) Da[k] *= rho * vm[k % 3];
    addToQuadrant(B, Da, 1, 1);
  }
  if (symmetric) {                        // mju_symmetrize (engine_util_blas.c:794-801)
    for (int r = 0; r < 6; r++) {
      for (int k = 0; k < r; k++) B[r*6+k] = B[k*6+r] = 0.5 * (B[r*6+k] + B[k*6+r]);
    }
  }
}

// the local 6 x nv Jacobian of a frame into Dtmp (rotation rows, then translation): mj_jac at
// `point`, each half rotated by mju_mulMatTMat(xmat, ., 3, 3, nv) (engine_util_blas.c:884-897,
// zero entries of xmat skipped)
template <int S, class P, class X>
MJH_HD void localJac(const mjhipModel& m, const Lane<S>& d, P point, X xmat, int body) {
  const int nv = m.nv;
  jacInto(m, d, d.jacp, d.jacr, point, body);
  double R[9];
  for (int k = 0; k < 9; k++) R[k] = xmat[k];
  for (int h = 0; h < 2; h++) {
    SP<S> src = h ? d.jacp : d.jacr;
    SP<S> dst = d.Dtmp + 3*h*nv;
    for (int k = 0; k < nv; k++) {
      const double v0 = src[k], v1 = src[nv + k], v2 = src[2*nv + k];
      for (int j = 0; j < 3; j++) {
        double t = 0;
        if (R[j]) t += v0*R[j];
        if (R[3 + j]) t += v1*R[3 + j];
        if (R[6 + j]) t += v2*R[6 + j];
        dst[j*nv + k] = t;
      }
    }
  }
}

// mjd_passive_vel :1494-1513: qDeriv += the fluid models' d qfrc_fluid / d qvel
// (mjd_ellipsoidFluid :1168-1270, mjd_inertiaBoxFluid :1275-1425, dense Jacobians)
template <int S>
MJH_HD void fluidDeriv(const mjhipModel& m, const Lane<S>& d) {
  const int nv = m.nv;
  const double rho = m.opt.density, mu = m.opt.viscosity;
  for (int i = 1; i < m.nbody; i++) {
    if (m.body_mass[i] < MINVAL) continue;
    int ell = 0;
    for (int j = 0; j < m.body_geomnum[i] && ell == 0; j++) {
      ell += m.geom_fluid[12*(m.body_geomadr[i] + j)] > 0;
    }
    double lvel[6], wind[6], lwind[6];
    for (int k = 0; k < 3; k++) { wind[k] = 0; wind[3 + k] = m.opt.wind[k]; }
    if (ell) {
      for (int j = 0; j < m.body_geomnum[i]; j++) {
        const int g = m.body_geomadr[i] + j;
        const double* c = m.geom_fluid + 12*g;
        const double* sz = m.geom_size + 3*g;
        double ax[3], B[36];                // mju_geomSemiAxes (engine_util_misc.c:425-451)
        const int t = m.geom_type[g];
        if (t == mjhipGEOM_SPHERE) { ax[0] = sz[0]; ax[1] = sz[0]; ax[2] = sz[0]; }
        else if (t == mjhipGEOM_CAPSULE) { ax[0] = sz[0]; ax[1] = sz[0]; ax[2] = sz[1] + sz[0]; }
        else if (t == mjhipGEOM_CYLINDER) { ax[0] = sz[0]; ax[1] = sz[0]; ax[2] = sz[1]; }
        else { ax[0] = sz[0]; ax[1] = sz[1]; ax[2] = sz[2]; }
        if (c[0] == 0.0) continue;
        objectVelocity(m, d, 5, g, lvel, 1);   // mjOBJ_GEOM
        transformSpatial(lwind, wind, 0, d.geom_xpos + 3*g, d.subtree_com + 3*m.body_rootid[i],
                         d.geom_xmat + 9*g, true);
        lvel[3] -= lwind[3]; lvel[4] -= lwind[4]; lvel[5] -= lwind[5];
        localJac(m, d, d.geom_xpos + 3*g, d.geom_xmat + 9*g, m.geom_bodyid[g]);
        ellipsoidFluidB(B, lvel, rho, mu, ax, c, m.opt.integrator == mjhipINT_IMPLICITFAST);
        addJTBJ(m, d, d.Dtmp, B, 6);
      }
      continue;
    }
    const double* inertia = m.body_inertia + 3*i;
    const double mass = m.body_mass[i];
    auto mx = [](double a, double b) { return a > b ? a : b; };
    double box[3], B;
    box[0] = sqrt(mx(MINVAL, (inertia[1] + inertia[2] - inertia[0])) / mass * 6.0);
    box[1] = sqrt(mx(MINVAL, (inertia[0] + inertia[2] - inertia[1])) / mass * 6.0);
    box[2] = sqrt(mx(MINVAL, (inertia[0] + inertia[1] - inertia[2])) / mass * 6.0);
    objectVelocity(m, d, 1, i, lvel, 1);
    transformSpatial(lwind, wind, 0, d.xipos + 3*i, d.subtree_com + 3*m.body_rootid[i],
                     d.ximat + 9*i, true);
    lvel[3] -= lwind[3]; lvel[4] -= lwind[4]; lvel[5] -= lwind[5];
    localJac(m, d, d.xipos + 3*i, d.ximat + 9*i, i);
    SP<S> J = d.Dtmp;
    if (mu > 0) {
      const double diam = (box[0] + box[1] + box[2])/3.0;
      B = -mjhipPI*diam*diam*diam*mu;
      for (int j = 0; j < 3; j++) addJTBJ(m, d, J + j*nv, &B, 1);
      B = -3.0*mjhipPI*diam*mu;
      for (int j = 0; j < 3; j++) addJTBJ(m, d, J + 3*nv + j*nv, &B, 1);
    }
    if (rho > 0) {
      B = -rho*box[0]*(box[1]*box[1]*box[1]*box[1]+box[2]*box[2]*box[2]*box[2])*
          2*fabs(lvel[0])/64.0;
      addJTBJ(m, d, J, &B, 1);
      B = -rho*box[1]*(box[0]*box[0]*box[0]*box[0]+box[2]*box[2]*box[2]*box[2])*
          2*fabs(lvel[1])/64.0;
      addJTBJ(m, d, J + nv, &B, 1);
      B = -rho*box[2]*(box[0]*box[0]*box[0]*box[0]+box[1]*box[1]*box[1]*box[1])*
          2*fabs(lvel[2])/64.0;
      addJTBJ(m, d, J + 2*nv, &B, 1);
      B = -0.5*rho*box[1]*box[2]*2*fabs(lvel[3]);
      addJTBJ(m, d, J + 3*nv, &B, 1);
      B = -0.5*rho*box[0]*box[2]*2*fabs(lvel[4]);
      addJTBJ(m, d, J + 4*nv, &B, 1);
      B = -0.5*rho*box[0]*box[1]*2*fabs(lvel[5]);
      addJTBJ(m, d, J + 5*nv, &B, 1);
    }
  }
}

// address of (r, c) in the D sparsity (c an ancestor of r: the inverse of mapD2M)
MJH_HD int dAdr(const mjhipModel& m, int r, int c) {
  const int adr = m.D_rowadr[r];
  int k = 0;
  while (k < m.D_rownnz[r] - 1 && m.D_colind[adr + k] != c) k++;
  return adr + k;
}

// mj_discreteAcc engine_inverse.c:81-164:
//   Euler: qacc <- M^-1 (M + h*diag(B)) qacc when implicit damping applies
//   implicitfast: qacc <- M^-1 (M - h*qDeriv) qacc, qDeriv reduced to qM's sparsity; the
//   modified M entries are formed on the fly (same values as the reference's in-place qM)
//   implicit: qacc <- M^-1 (M - h*qDeriv) qacc, the full qDeriv (incl. mjd_rne_vel) on the D
//   sparsity (the reference's qLU before its factorization)
template <int S>
MJH_HD void discreteAcc(const mjhipModel& m, const Lane<S>& d) {
  const int nv = m.nv;
  if (m.opt.integrator == mjhipINT_IMPLICIT) {
    // mjd_smooth_vel(flg_bias = 1) on the D sparsity; qLU = qM (mapM2D) - h*qDeriv;
    // qfrc = qLU*qacc (mju_mulMatVecSparse engine_util_sparse.c:156-166)
    for (int r = 0; r < nv; r++) {
      const int adr = m.D_rowadr[r];
      for (int k = 0; k < m.D_rownnz[r]; k++) {
        d.qDeriv[adr + k] = qDerivAt(m, d, r, m.D_colind[adr + k]);
      }
    }
    if (mjh_fluidDeriv(&m)) fluidDeriv(m, d);
    rneVel(m, d);
    for (int i = 0; i < m.nD; i++) {
      d.qLU[i] = d.qM[m.mapM2D[i]] + d.qDeriv[i] * -m.opt.timestep;
    }
    for (int r = 0; r < nv; r++) {
      const int adr = m.D_rowadr[r];
      d.qforce[r] = dotSparse(d.qLU + adr, d.qacc, m.D_rownnz[r], m.D_colind + adr);
    }
    copy(d.qacc, d.qforce, nv);
    solveM(m, d, d.qacc);
    return;
  }
  if (m.opt.integrator == mjhipINT_IMPLICITFAST && mjh_fluidDeriv(&m)) {
    // mjd_smooth_vel(flg_bias = 0) on the D sparsity with the fluid terms, then mj_mulM with
    // qM + qDeriv*(-h) reduced to qM's sparsity
    for (int r = 0; r < nv; r++) {
      const int adr = m.D_rowadr[r];
      for (int k = 0; k < m.D_rownnz[r]; k++) {
        d.qDeriv[adr + k] = qDerivAt(m, d, r, m.D_colind[adr + k]);
      }
    }
    fluidDeriv(m, d);
    const double h = m.opt.timestep;
    for (int i = 0; i < nv; i++) {
      int adr = m.dof_Madr[i];
      d.qforce[i] = (d.qM[adr] + d.qDeriv[dAdr(m, i, i)] * -h)*d.qacc[i];
      if (m.dof_simplenum[i]) continue;
      int j = m.dof_parentid[i];
      while (j >= 0) {
        adr++;
        double Mij = d.qM[adr] + d.qDeriv[dAdr(m, i, j)] * -h;
        d.qforce[i] += Mij*d.qacc[j];
        d.qforce[j] += Mij*d.qacc[i];
        j = m.dof_parentid[j];
      }
    }
    copy(d.qacc, d.qforce, nv);
    solveM(m, d, d.qacc);
    return;
  }
  if (m.opt.integrator == mjhipINT_IMPLICITFAST) {
    const double h = m.opt.timestep;
    zero(d.qforce, nv);
    for (int i = 0; i < nv; i++) {          // mj_mulM with qM + qDeriv*(-h)
      int adr = m.dof_Madr[i];
      d.qforce[i] = (d.qM[adr] + qDerivAt(m, d, i, i) * -h)*d.qacc[i];
      if (m.dof_simplenum[i]) continue;
      int j = m.dof_parentid[i];
      while (j >= 0) {
        adr++;
        double Mij = d.qM[adr] + qDerivAt(m, d, i, j) * -h;
        d.qforce[i] += Mij*d.qacc[j];
        d.qforce[j] += Mij*d.qacc[i];
        j = m.dof_parentid[j];
      }
    }
    copy(d.qacc, d.qforce, nv);
    solveM(m, d, d.qacc);
    return;
  }
  int dof_damping = 0;
  if (!(m.opt.disableflags & mjhipDSBL_EULERDAMP)) {
    for (int i = 0; i < nv; i++) {
      if (m.dof_damping[i] > 0) {
        dof_damping = 1;
        break;
      }
    }
  }
  if (!dof_damping) return;
  mulM(m, d, d.qforce, d.qacc);
  for (int i = 0; i < nv; i++) d.qforce[i] += m.opt.timestep * m.dof_damping[i] * d.qacc[i];
  copy(d.qacc, d.qforce, nv);
  solveM(m, d, d.qacc);
}

//---------------------------------- engine_sensor.c (energy) ---------------------------------

// mj_energyPos engine_sensor.c:920-1008 (no flex): gravity, joint and tendon springs. As the
// reference, the free joint's translational term normalizes (x, y, z, qw) as a quaternion
// before differencing, and the ball term differences the raw qpos quaternion.
template <int S>
MJH_HD void energyPos(const mjhipModel& m, const Lane<S>& d) {
  double e = 0, dif[3];
  if (!(m.opt.disableflags & mjhipDSBL_GRAVITY)) {
    const double* g = m.opt.gravity;
    for (int i = 1; i < m.nbody; i++) {
      SP<S> x = d.xipos + 3*i;
      e -= m.body_mass[i] * (g[0]*x[0] + g[1]*x[1] + g[2]*x[2]);
    }
  }
  if (!(m.opt.disableflags & mjhipDSBL_PASSIVE)) {
    for (int i = 0; i < m.njnt; i++) {
      const double k = m.jnt_stiffness[i];
      int padr = m.jnt_qposadr[i];
      const int t = m.jnt_type[i];
      if (t == mjhipJNT_FREE || t == mjhipJNT_BALL) {
        if (t == mjhipJNT_FREE) {
          double quat[4] = {d.qpos[padr], d.qpos[padr+1], d.qpos[padr+2], d.qpos[padr+3]};
          normalize4(quat);
          sub3(dif, quat, m.qpos_spring + padr);
          e += 0.5*k*(dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2]);
          padr += 3;
        }
        subQuat(dif, d.qpos + padr, m.qpos_spring + padr);
        e += 0.5*k*(dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2]);
      } else {
        const double x = d.qpos[padr] - m.qpos_spring[padr];
        e += 0.5*k*x*x;
      }
    }
    for (int i = 0; i < m.ntendon; i++) {
      const double len = d.ten_length[i];
      const double lo = m.tendon_lengthspring[2*i], hi = m.tendon_lengthspring[2*i+1];
      double disp = 0;
      if (len > hi) disp = hi - len;
      else if (len < lo) disp = lo - len;
      e += 0.5*m.tendon_stiffness[i]*disp*disp;
    }
  }
  d.energy[0] = e;
}

// mj_energyVel engine_sensor.c:1011-1020: 0.5 qvel' M qvel
template <int S>
MJH_HD void energyVel(const mjhipModel& m, const Lane<S>& d) {
  mulM(m, d, d.qforce, d.qvel);
  d.energy[1] = 0.5*dot(d.qforce, d.qvel, m.nv);
}

//---------------------------------- engine_sensor.c (sensors) ------------------------------

// engine_util_blas.c:179-188
template <class R, class M, class V> MJH_HD void mulMatTVec3(R res, M mat, V vec) {
  const double t0 = mat[0]*vec[0] + mat[3]*vec[1] + mat[6]*vec[2];
  const double t1 = mat[1]*vec[0] + mat[4]*vec[1] + mat[7]*vec[2];
  const double t2 = mat[2]*vec[0] + mat[5]*vec[1] + mat[8]*vec[2];
  res[0] = t0; res[1] = t1; res[2] = t2;
}

// engine_util_spatial.c:495-523; rot may be null (no rotation)
template <class R, class V, class P, class O, class M>
MJH_HD void transformSpatial(R res, V vec, int flg_force, P newpos, O oldpos, M rot,
                             bool has_rot) {
  double cros[3], dif[3], tran[6];
  for (int i = 0; i < 6; i++) tran[i] = vec[i];
  sub3(dif, newpos, oldpos);
  if (flg_force) {
    double f[3] = {vec[3], vec[4], vec[5]};
    cross(cros, dif, f);
    double t[3] = {vec[0], vec[1], vec[2]};
    sub3(tran, t, cros);
  } else {
    double w[3] = {vec[0], vec[1], vec[2]};
    cross(cros, dif, w);
    double t[3] = {vec[3], vec[4], vec[5]};
    sub3(tran + 3, t, cros);
  }
  if (has_rot) {
    mulMatTVec3(res, rot, tran);
    double r[3];
    mulMatTVec3(r, rot, tran + 3);
    res[3] = r[0]; res[4] = r[1]; res[5] = r[2];
  } else {
    for (int i = 0; i < 6; i++) res[i] = tran[i];
  }
}

// frame (pos, rot) and body of a sensorized object (mjtObj body/xbody/geom/site/camera):
// the switch of mj_objectVelocity (engine_support.c:1265-1312) and get_xpos_xmat
// (engine_sensor.c:69-94)
template <int S>
MJH_HD int objFrame(const mjhipModel& m, const Lane<S>& d, int type, int id, SP<S>& pos,
                    SP<S>& mat) {
  switch (type) {
  case 1: pos = d.xipos + 3*id; mat = d.ximat + 9*id; return id;
  case 2: pos = d.xpos + 3*id; mat = d.xmat + 9*id; return id;
  case 5: pos = d.geom_xpos + 3*id; mat = d.geom_xmat + 9*id; return m.geom_bodyid[id];
  case 6: pos = d.site_xpos + 3*id; mat = d.site_xmat + 9*id; return m.site_bodyid[id];
  default: pos = d.cam_xpos + 3*id; mat = d.cam_xmat + 9*id; return m.cam_bodyid[id];
  }
}

// engine_support.c:1265-1312
template <int S, class R>
MJH_HD void objectVelocity(const mjhipModel& m, const Lane<S>& d, int type, int id, R res,
                           int flg_local) {
  SP<S> pos, mat;
  const int b = objFrame(m, d, type, id, pos, mat);
  transformSpatial(res, d.cvel + 6*b, 0, pos, d.subtree_com + 3*m.body_rootid[b], mat,
                   flg_local != 0);
}

// engine_support.c:1317-1371
template <int S, class R>
MJH_HD void objectAcceleration(const mjhipModel& m, const Lane<S>& d, int type, int id, R res,
                               int flg_local) {
  SP<S> pos, mat;
  double correction[3], vel[6];
  const int b = objFrame(m, d, type, id, pos, mat);
  SP<S> com = d.subtree_com + 3*m.body_rootid[b];
  transformSpatial(vel, d.cvel + 6*b, 0, pos, com, mat, flg_local != 0);
  transformSpatial(res, d.cacc + 6*b, 0, pos, com, mat, flg_local != 0);
  cross(correction, vel, vel + 3);
  res[3] += correction[0]; res[4] += correction[1]; res[5] += correction[2];
}

// engine_sensor.c:96-118 get_xquat
template <int S>
MJH_HD void objQuat(const mjhipModel& m, const Lane<S>& d, int type, int id, double q[4]) {
  switch (type) {
  case 2: copy4(q, d.xquat + 4*id); break;
  case 1: mulQuat(q, d.xquat + 4*id, m.body_iquat + 4*id); break;
  case 5: mulQuat(q, d.xquat + 4*m.geom_bodyid[id], m.geom_quat + 4*id); break;
  case 6: mulQuat(q, d.xquat + 4*m.site_bodyid[id], m.site_quat + 4*id); break;
  default: mulQuat(q, d.xquat + 4*m.cam_bodyid[id], m.cam_quat + 4*id); break;
  }
}

// engine_core_smooth.c:1900-1958
template <int S>
MJH_HD void subtreeVel(const mjhipModel& m, const Lane<S>& d) {
  const int nbody = m.nbody;
  double dx[3], dv[3], dp[3], dL[3];
  for (int i = 0; i < nbody; i++) {
    double bv[6];
    objectVelocity(m, d, 1, i, bv, 0);
    for (int k = 0; k < 6; k++) d.body_vel[6*i + k] = bv[k];
    scl3(d.subtree_linvel + 3*i, bv + 3, m.body_mass[i]);
    mulMatTVec3(dv, d.ximat + 9*i, bv);
    dv[0] *= m.body_inertia[3*i];
    dv[1] *= m.body_inertia[3*i+1];
    dv[2] *= m.body_inertia[3*i+2];
    mulMatVec3(d.subtree_angmom + 3*i, d.ximat + 9*i, dv);
  }
  for (int i = nbody-1; i >= 0; i--) {
    if (i) addTo3(d.subtree_linvel + 3*m.body_parentid[i], d.subtree_linvel + 3*i);
    const double sm = m.body_subtreemass[i];
    scl3(d.subtree_linvel + 3*i, d.subtree_linvel + 3*i, 1/(sm > MINVAL ? sm : MINVAL));
  }
  for (int i = nbody-1; i > 0; i--) {
    const int parent = m.body_parentid[i];
    sub3(dx, d.xipos + 3*i, d.subtree_com + 3*i);
    sub3(dv, d.body_vel + 6*i + 3, d.subtree_linvel + 3*i);
    scl3(dp, dv, m.body_mass[i]);
    cross(dL, dx, dp);
    addTo3(d.subtree_angmom + 3*i, dL);
    addTo3(d.subtree_angmom + 3*parent, d.subtree_angmom + 3*i);
    sub3(dx, d.subtree_com + 3*i, d.subtree_com + 3*parent);
    sub3(dv, d.subtree_linvel + 3*i, d.subtree_linvel + 3*parent);
    scl3(dv, dv, m.body_subtreemass[i]);
    cross(dL, dx, dv);
    addTo3(d.subtree_angmom + 3*parent, dL);
  }
}

// engine_core_smooth.c:2027-2181 mj_rnePostConstraint: cacc, cfrc_int, cfrc_ext (contact
// forces via mj_contactForce / mju_decodePyramid, engine_support.c:1459-1480,
// engine_util_misc.c:830-850; no equality constraints in the supported subset)
template <int S>
MJH_HD void rnePostConstraint(const mjhipModel& m, const Lane<S>& d) {
  const int nbody = m.nbody;
  double cfrc_com[6], cfrc[6], lfrc[6];
  zero(d.cacc, 6);
  if (!(m.opt.disableflags & mjhipDSBL_GRAVITY)) {
    d.cacc[3] = m.opt.gravity[0]*-1; d.cacc[4] = m.opt.gravity[1]*-1;
    d.cacc[5] = m.opt.gravity[2]*-1;
  }
  zero(d.cfrc_ext, 6*nbody);
  for (int i = 1; i < nbody; i++) {
    SP<S> xf = d.xfrc_applied + 6*i;
    bool nz = false;
    for (int k = 0; k < 6; k++) nz |= (xf[k] != 0);
    if (nz) {
      cfrc[0] = xf[3]; cfrc[1] = xf[4]; cfrc[2] = xf[5];
      cfrc[3] = xf[0]; cfrc[4] = xf[1]; cfrc[5] = xf[2];
      transformSpatial(cfrc_com, cfrc, 1, d.subtree_com + 3*m.body_rootid[i], d.xipos + 3*i,
                       cfrc, false);
      addTo(d.cfrc_ext + 6*i, cfrc_com, 6);
    }
  }
  const int ncon = d.con_cap ? d.con_count[0] : 0;
  for (int i = 0; i < ncon; i++) {
    const int adr = d.con_efc_address[i];
    const int g0 = d.con_geom[2*i], g1 = d.con_geom[2*i + 1];
    if (adr < 0 || g0 < 0 || g1 < 0) continue;
    zero(lfrc, 6);
    const int dim = d.con_dim[i];
    if (m.opt.cone == mjhipCONE_ELLIPTIC) {        // mj_contactForce: the cone's own force
      for (int k = 0; k < dim; k++) lfrc[k] = d.efc_force[adr + k];
    } else if (dim == 1) {
      lfrc[0] = d.efc_force[adr];
    } else {
      lfrc[0] = 0;
      for (int k = 0; k < 2*(dim-1); k++) lfrc[0] += d.efc_force[adr + k];
      for (int k = 0; k < dim-1; k++) {
        lfrc[k+1] = (d.efc_force[adr + 2*k] - d.efc_force[adr + 2*k + 1]) * d.con_friction[5*i + k];
      }
    }
    auto frame = d.con_frame + 9*i;
    mulMatTVec3(cfrc, frame, lfrc + 3);
    double t[3];
    mulMatTVec3(t, frame, lfrc);
    cfrc[3] = t[0]; cfrc[4] = t[1]; cfrc[5] = t[2];
    int k;
    if ((k = m.geom_bodyid[g0])) {
      transformSpatial(cfrc_com, cfrc, 1, d.subtree_com + 3*m.body_rootid[k], d.con_pos + 3*i,
                       cfrc, false);
      subFrom(d.cfrc_ext + 6*k, cfrc_com, 6);
    }
    if ((k = m.geom_bodyid[g1])) {
      transformSpatial(cfrc_com, cfrc, 1, d.subtree_com + 3*m.body_rootid[k], d.con_pos + 3*i,
                       cfrc, false);
      addTo(d.cfrc_ext + 6*k, cfrc_com, 6);
    }
  }
  // connect and weld forces (:2102-2158); joint/tendon rows apply no body force
  const int ne = d.efc_count[1];
  for (int i = 0; i < ne;) {
    const int id = d.efc_id[i], t = m.eq_type[id];
    if (t != mjhipEQ_CONNECT && t != mjhipEQ_WELD) {
      i++;
      continue;
    }
    const double* eq_data = m.eq_data + mjhipNEQDATA*id;
    cfrc[3] = d.efc_force[i]; cfrc[4] = d.efc_force[i+1]; cfrc[5] = d.efc_force[i+2];
    if (t == mjhipEQ_WELD) {
      cfrc[0] = d.efc_force[i+3]; cfrc[1] = d.efc_force[i+4]; cfrc[2] = d.efc_force[i+5];
    } else {
      cfrc[0] = 0; cfrc[1] = 0; cfrc[2] = 0;
    }
    const bool body_semantic = m.eq_objtype[id] == 1;
    for (int side = 0; side < 2; side++) {
      const int obj = side ? m.eq_obj2id[id] : m.eq_obj1id[id];
      const int k = body_semantic ? obj : m.site_bodyid[obj];
      if (!k) continue;
      const int sel = side ? (t == mjhipEQ_CONNECT) : (t == mjhipEQ_WELD);
      const double* offset = body_semantic ? eq_data + 3*sel : m.site_pos + 3*obj;
      double pos[3];
      mulMatVec3(pos, d.xmat + 9*k, offset);
      addTo3(pos, d.xpos + 3*k);
      transformSpatial(cfrc_com, cfrc, 1, d.subtree_com + 3*m.body_rootid[k], pos, cfrc, false);
      if (side) subFrom(d.cfrc_ext + 6*k, cfrc_com, 6);
      else addTo(d.cfrc_ext + 6*k, cfrc_com, 6);
    }
    i += t == mjhipEQ_WELD ? 6 : 3;
  }
  double cacc[6], cfrc_body[6], cfrc_corr[6];
  zero(d.cfrc_int, 6);
  for (int j = 1; j < nbody; j++) {
    const int bda = m.body_dofadr[j];
    mulDofVec(cacc, d.cdof_dot + 6*bda, d.qvel + bda, m.body_dofnum[j]);
    add(d.cacc + 6*j, d.cacc + 6*m.body_parentid[j], cacc, 6);
    mulDofVec(cacc, d.cdof + 6*bda, d.qacc + bda, m.body_dofnum[j]);
    addTo(d.cacc + 6*j, cacc, 6);
    mulInertVec(cfrc_body, d.cinert + 10*j, d.cacc + 6*j);
    mulInertVec(cfrc_corr, d.cinert + 10*j, d.cvel + 6*j);
    crossForce(cfrc, d.cvel + 6*j, cfrc_corr);
    addTo(cfrc_body, cfrc, 6);
    for (int k = 0; k < 6; k++) d.cfrc_int[6*j + k] = cfrc_body[k] - d.cfrc_ext[6*j + k];
  }
  for (int j = nbody-1; j > 0; j--) {
    addTo(d.cfrc_int + 6*m.body_parentid[j], d.cfrc_int + 6*j, 6);
  }
}

// engine_sensor.c:38-66
template <int S>
MJH_HD void applyCutoff(const mjhipModel& m, const Lane<S>& d, int stage) {
  for (int i = 0; i < m.nsensor; i++) {
    if (m.sensor_needstage[i] == stage && m.sensor_cutoff[i] > 0) {
      if (m.sensor_type[i] == mjhSENS_GEOMFROMTO) continue;   // :44-47
      const int adr = m.sensor_adr[i], dim = m.sensor_dim[i];
      const double cutoff = m.sensor_cutoff[i];
      for (int j = 0; j < dim; j++) {
        const double x = d.sensordata[adr + j];
        if (m.sensor_datatype[i] == 0) {
          d.sensordata[adr + j] = x < -cutoff ? -cutoff : (x > cutoff ? cutoff : x);
        } else if (m.sensor_datatype[i] == 1) {
          d.sensordata[adr + j] = cutoff < x ? cutoff : x;
        }
      }
    }
  }
}

// first limit row of (type, id) among rows ne+nf..nefc (engine_sensor.c:286-304); -1 if none
template <int S>
MJH_HD int limitRow(const Lane<S>& d, int type, int id) {
  const int nefc = d.efc_count[0], start = d.efc_count[1] + d.efc_count[2];
  for (int j = start; j < nefc; j++) {
    if (d.efc_type[j] == type && d.efc_id[j] == id) return j;
  }
  return -1;
}

// engine_sensor.c:126-215 cam_project (the oracle's or_camProject): the reference's explicit
// 4x4 product image * focal * rotation * translation, every term in its loop order
template <class Q, class P, class M>
MJH_HD void camProject(double out[2], Q target, P cpos, M cmat, const int* res, double fovy,
                       const float* intr, const float* size) {
  double T[4][4] = {{0}}, Rm[4][4] = {{0}}, F[3][4] = {{0}}, I[3][3] = {{0}}, Pm[3][4] = {{0}};
  double fx, fy;
  for (int i = 0; i < 4; i++) T[i][i] = Rm[i][i] = 1;
  for (int i = 0; i < 3; i++) T[i][3] = -cpos[i];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) Rm[i][j] = cmat[3*j+i];
  }
  if (size[0] && size[1]) {
    fx = intr[0] / size[0] * res[0];
    fy = intr[1] / size[1] * res[1];
  } else {
    fx = fy = .5 / tan(fovy * mjhipPI / 360.) * res[1];
  }
  F[0][0] = -fx;
  F[1][1] = fy;
  F[2][2] = 1.0;
  I[0][0] = I[1][1] = I[2][2] = 1;
  I[0][2] = (double)res[0] / 2.0;
  I[1][2] = (double)res[1] / 2.0;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      for (int k = 0; k < 4; k++)
        for (int l = 0; l < 4; l++)
          for (int n = 0; n < 4; n++) Pm[i][n] += I[i][j] * F[j][k] * Rm[k][l] * T[l][n];
  const double ph[4] = {target[0], target[1], target[2], 1};
  double px[3] = {0, 0, 0};
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 4; j++) px[i] += Pm[i][j] * ph[j];
  }
  double den = px[2];
  if (fabs(den) < MINVAL) den = den < 0 ? dmin(den, -MINVAL) : dmax(den, MINVAL);
  out[0] = px[0] / den;
  out[1] = px[1] / den;
}

// mj_ray for the rangefinder (defined with the touch sensor's ray functions below)
template <int S>
MJH_HD double ray(const mjhipModel& m, const Lane<S>& d, const double pnt[3],
                  const double vec[3], int bodyexclude);

// engine_sensor.c:209-513 mj_sensorPos (no user/plugin sensors, rejected at load)
template <int S>
MJH_HD void sensorPos(const mjhipModel& m, const Lane<S>& d) {
  if (m.opt.disableflags & mjhipDSBL_SENSOR) return;
  for (int i = 0; i < m.nsensor; i++) {
    if (m.sensor_needstage[i] != mjhipSTAGE_POS) continue;
    const int type = m.sensor_type[i], objtype = m.sensor_objtype[i];
    const int objid = m.sensor_objid[i], refid = m.sensor_refid[i];
    const int reftype = m.sensor_reftype[i];
    SP<S> out = d.sensordata + m.sensor_adr[i];
    SP<S> xpos, xmat, xpos_ref, xmat_ref;
    double rvec[3];
    int r;
    switch (type) {
    case mjhSENS_MAGNETOMETER:
      mulMatTVec(out, d.site_xmat + 9*objid, m.opt.magnetic, 3, 3);
      break;
    case mjhSENS_GEOMDIST:
    case mjhSENS_GEOMNORMAL:
    case mjhSENS_GEOMFROMTO: {
      // engine_sensor.c:378-460: the smallest distance over the two bodies'/geoms' geom
      // pairs, cutoff as the bound (the reference shares one evaluation among consecutive
      // sensors of the same pair and cutoff; recomputing gives the same values)
      const double margin = m.sensor_cutoff[i];
      double dist = margin, fromto[6] = {0, 0, 0, 0, 0, 0};
      const int n1 = objtype == 1 ? m.body_geomnum[objid] : 1;
      const int id1 = objtype == 1 ? m.body_geomadr[objid] : objid;
      const int n2 = reftype == 1 ? m.body_geomnum[refid] : 1;
      const int id2 = reftype == 1 ? m.body_geomadr[refid] : refid;
      int unused = 0;
      for (int a = id1; a < id1 + n1; a++) {
        for (int b = id2; b < id2 + n2; b++) {
          double ft[6];
          const double dn = geomDistance(m, d, a, b, margin, ft, &unused);
          if (dn < dist) {
            dist = dn;
            for (int k = 0; k < 6; k++) fromto[k] = ft[k];
          }
        }
      }
      if (type == mjhSENS_GEOMDIST) {
        out[0] = dist;
      } else if (type == mjhSENS_GEOMNORMAL) {
        double nrm[3] = {fromto[3]-fromto[0], fromto[4]-fromto[1], fromto[5]-fromto[2]};
        if (nrm[0] || nrm[1] || nrm[2]) normalize3(nrm);
        for (int k = 0; k < 3; k++) out[k] = nrm[k];
      } else {
        for (int k = 0; k < 6; k++) out[k] = fromto[k];
      }
      break;
    }
    case mjhSENS_CAMPROJECTION: {
      double px[2];
      camProject(px, d.site_xpos + 3*objid, d.cam_xpos + 3*refid, d.cam_xmat + 9*refid,
                 m.cam_resolution + 2*refid, m.cam_fovy[refid], m.cam_intrinsic + 4*refid,
                 m.cam_sensorsize + 2*refid);
      out[0] = px[0];
      out[1] = px[1];
      break;
    }
    case mjhSENS_RANGEFINDER:              // the site's z axis, its own body excluded
      rvec[0] = d.site_xmat[9*objid+2];
      rvec[1] = d.site_xmat[9*objid+5];
      rvec[2] = d.site_xmat[9*objid+8];
      {
        double pnt[3];
        for (int k = 0; k < 3; k++) pnt[k] = d.site_xpos[3*objid+k];
        out[0] = ray(m, d, pnt, rvec, m.site_bodyid[objid]);
      }
      break;
    case mjhSENS_JOINTPOS: out[0] = d.qpos[m.jnt_qposadr[objid]]; break;
    case mjhSENS_TENDONPOS: out[0] = d.ten_length[objid]; break;
    case mjhSENS_ACTUATORPOS: out[0] = d.actuator_length[objid]; break;
    case mjhSENS_BALLQUAT: {
      double q[4];
      copy4(q, d.qpos + m.jnt_qposadr[objid]);
      normalize4(q);
      copy4(out, q);
      break;
    }
    case mjhSENS_JOINTLIMITPOS:
    case mjhSENS_TENDONLIMITPOS:
      out[0] = 0;
      r = limitRow(d, type == mjhSENS_JOINTLIMITPOS ? CNSTR_LIMIT_JOINT : CNSTR_LIMIT_TENDON,
                   objid);
      if (r >= 0) out[0] = d.efc_pos[r] - d.efc_margin[r];
      break;
    case mjhSENS_FRAMEPOS:
    case mjhSENS_FRAMEXAXIS:
    case mjhSENS_FRAMEYAXIS:
    case mjhSENS_FRAMEZAXIS:
      objFrame(m, d, objtype, objid, xpos, xmat);
      if (refid == -1) {
        if (type == mjhSENS_FRAMEPOS) {
          copy3(out, xpos);
        } else {
          const int off = type - mjhSENS_FRAMEXAXIS;
          out[0] = xmat[off]; out[1] = xmat[off + 3]; out[2] = xmat[off + 6];
        }
      } else {
        objFrame(m, d, reftype, refid, xpos_ref, xmat_ref);
        if (type == mjhSENS_FRAMEPOS) {
          sub3(rvec, xpos, xpos_ref);
          mulMatTVec3(out, xmat_ref, rvec);
        } else {
          const int off = type - mjhSENS_FRAMEXAXIS;
          double axis[3] = {xmat[off], xmat[off + 3], xmat[off + 6]};
          mulMatTVec3(out, xmat_ref, axis);
        }
      }
      break;
    case mjhSENS_FRAMEQUAT: {
      double objquat[4], refquat[4], q[4];
      objQuat(m, d, objtype, objid, objquat);
      if (refid == -1) {
        copy4(out, objquat);
      } else {
        objQuat(m, d, reftype, refid, refquat);
        refquat[1] = -refquat[1]; refquat[2] = -refquat[2]; refquat[3] = -refquat[3];
        mulQuat(q, refquat, objquat);
        copy4(out, q);
      }
      break;
    }
    case mjhSENS_SUBTREECOM: copy3(out, d.subtree_com + 3*objid); break;
    case mjhSENS_E_POTENTIAL: energyPos(m, d); out[0] = d.energy[0]; break;
    case mjhSENS_E_KINETIC: energyVel(m, d); out[0] = d.energy[1]; break;
    case mjhSENS_CLOCK: out[0] = d.time[0]; break;
    default: break;
    }
  }
  applyCutoff(m, d, mjhipSTAGE_POS);
}

// engine_sensor.c:521-672 mj_sensorVel
template <int S>
MJH_HD void sensorVel(const mjhipModel& m, const Lane<S>& d) {
  if (m.opt.disableflags & mjhipDSBL_SENSOR) return;
  bool subtree = false;
  double xvel[6];
  for (int i = 0; i < m.nsensor; i++) {
    if (m.sensor_needstage[i] != mjhipSTAGE_VEL) continue;
    const int type = m.sensor_type[i], objtype = m.sensor_objtype[i];
    const int objid = m.sensor_objid[i], refid = m.sensor_refid[i];
    const int reftype = m.sensor_reftype[i];
    SP<S> out = d.sensordata + m.sensor_adr[i];
    int r;
    if (!subtree && (type == mjhSENS_SUBTREELINVEL || type == mjhSENS_SUBTREEANGMOM)) {
      subtreeVel(m, d);
      subtree = true;
    }
    switch (type) {
    case mjhSENS_VELOCIMETER:
      objectVelocity(m, d, 6, objid, xvel, 1);
      copy3(out, xvel + 3);
      break;
    case mjhSENS_GYRO:
      objectVelocity(m, d, 6, objid, xvel, 1);
      copy3(out, xvel);
      break;
    case mjhSENS_JOINTVEL: out[0] = d.qvel[m.jnt_dofadr[objid]]; break;
    case mjhSENS_TENDONVEL: out[0] = d.ten_velocity[objid]; break;
    case mjhSENS_ACTUATORVEL: out[0] = d.actuator_velocity[objid]; break;
    case mjhSENS_BALLANGVEL: copy3(out, d.qvel + m.jnt_dofadr[objid]); break;
    case mjhSENS_JOINTLIMITVEL:
    case mjhSENS_TENDONLIMITVEL:
      out[0] = 0;
      r = limitRow(d, type == mjhSENS_JOINTLIMITVEL ? CNSTR_LIMIT_JOINT : CNSTR_LIMIT_TENDON,
                   objid);
      if (r >= 0) out[0] = d.efc_vel[r];
      break;
    case mjhSENS_FRAMELINVEL:
    case mjhSENS_FRAMEANGVEL:
      objectVelocity(m, d, objtype, objid, xvel, 0);
      if (refid > -1) {
        SP<S> xpos, xmat, xpos_ref, xmat_ref;
        double xvel_ref[6], rel_vel[6], crs[3], rvec[3];
        objFrame(m, d, objtype, objid, xpos, xmat);
        objFrame(m, d, reftype, refid, xpos_ref, xmat_ref);
        objectVelocity(m, d, reftype, refid, xvel_ref, 0);
        for (int k = 0; k < 6; k++) rel_vel[k] = xvel[k] - xvel_ref[k];
        sub3(rvec, xpos, xpos_ref);
        cross(crs, rvec, xvel_ref);
        addTo3(rel_vel + 3, crs);
        mulMatTVec3(xvel, xmat_ref, rel_vel);
        mulMatTVec3(xvel + 3, xmat_ref, rel_vel + 3);
      }
      copy3(out, type == mjhSENS_FRAMELINVEL ? xvel + 3 : xvel);
      break;
    case mjhSENS_SUBTREELINVEL: copy3(out, d.subtree_linvel + 3*objid); break;
    case mjhSENS_SUBTREEANGMOM: copy3(out, d.subtree_angmom + 3*objid); break;
    default: break;
    }
  }
  applyCutoff(m, d, mjhipSTAGE_VEL);
}

// engine_ray.c ray-zone tests for the touch sensor (mju_rayGeom :818-846 and the primitive
// intersections :37-445), on local copies of the zone's frame
MJH_HD void rayMap(const double* pos, const double* mat, const double* pnt, const double* vec,
                   double* lpnt, double* lvec) {
  const double dif[3] = {pnt[0]-pos[0], pnt[1]-pos[1], pnt[2]-pos[2]};
  lpnt[0] = mat[0]*dif[0] + mat[3]*dif[1] + mat[6]*dif[2];
  lpnt[1] = mat[1]*dif[0] + mat[4]*dif[1] + mat[7]*dif[2];
  lpnt[2] = mat[2]*dif[0] + mat[5]*dif[1] + mat[8]*dif[2];
  lvec[0] = mat[0]*vec[0] + mat[3]*vec[1] + mat[6]*vec[2];
  lvec[1] = mat[1]*vec[0] + mat[4]*vec[1] + mat[7]*vec[2];
  lvec[2] = mat[2]*vec[0] + mat[5]*vec[1] + mat[8]*vec[2];
}

MJH_HD double rayQuad(double a, double b, double c, double* x) {
  double det = b*b - a*c;
  if (det < MINVAL) {
    x[0] = -1;
    x[1] = -1;
    return -1;
  }
  det = sqrt(det);
  x[0] = (-b-det)/a;
  x[1] = (-b+det)/a;
  if (x[0] >= 0) return x[0];
  if (x[1] >= 0) return x[1];
  return -1;
}

MJH_HD double raySphere(const double* pos, double dist_sqr, const double* pnt,
                        const double* vec) {
  const double dif[3] = {pnt[0]-pos[0], pnt[1]-pos[1], pnt[2]-pos[2]};
  const double a = vec[0]*vec[0] + vec[1]*vec[1] + vec[2]*vec[2];
  const double b = vec[0]*dif[0] + vec[1]*dif[1] + vec[2]*dif[2];
  const double c = dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2] - dist_sqr;
  double xx[2];
  return rayQuad(a, b, c, xx);
}

MJH_HD double rayGeom(const double* pos, const double* mat, const double* size,
                      const double* pnt, const double* vec, int type) {
  double lpnt[3], lvec[3], xx[2], x = -1, sol;
  if (type == mjhipGEOM_SPHERE) return raySphere(pos, size[0]*size[0], pnt, vec);
  if (type == mjhipGEOM_CAPSULE) {
    const double ssz = size[0] + size[1];
    if (raySphere(pos, ssz*ssz, pnt, vec) < 0) return -1;
  } else if (type == mjhipGEOM_CYLINDER) {
    if (raySphere(pos, size[0]*size[0] + size[1]*size[1], pnt, vec) < 0) return -1;
  } else if (type == mjhipGEOM_BOX) {
    if (raySphere(pos, size[0]*size[0] + size[1]*size[1] + size[2]*size[2], pnt, vec) < 0) {
      return -1;
    }
  } else if (type != mjhipGEOM_PLANE && type != mjhipGEOM_ELLIPSOID) {
    return -1;
  }
  rayMap(pos, mat, pnt, vec, lpnt, lvec);
  if (type == mjhipGEOM_PLANE) {                        // ray_plane :191-218
    if (lvec[2] > -MINVAL) return -1;
    x = -lpnt[2]/lvec[2];
    if (x < 0) return -1;
    const double p0 = lpnt[0] + x*lvec[0], p1 = lpnt[1] + x*lvec[1];
    return ((size[0] <= 0 || fabs(p0) <= size[0]) && (size[1] <= 0 || fabs(p1) <= size[1]))
           ? x : -1;
  }
  if (type == mjhipGEOM_ELLIPSOID) {                    // ray_ellipsoid :305-323
    const double sx = 1/(size[0]*size[0]), sy = 1/(size[1]*size[1]), sz = 1/(size[2]*size[2]);
    const double a = sx*lvec[0]*lvec[0] + sy*lvec[1]*lvec[1] + sz*lvec[2]*lvec[2];
    const double b = sx*lvec[0]*lpnt[0] + sy*lvec[1]*lpnt[1] + sz*lvec[2]*lpnt[2];
    const double c = sx*lpnt[0]*lpnt[0] + sy*lpnt[1]*lpnt[1] + sz*lpnt[2]*lpnt[2] - 1;
    return rayQuad(a, b, c, xx);
  }
  if (type == mjhipGEOM_BOX) {                          // ray_box :387-445
    const int iface[3][2] = {{1, 2}, {0, 2}, {0, 1}};
    for (int i = 0; i < 3; i++) {
      if (fabs(lvec[i]) > MINVAL) {
        for (int side = -1; side <= 1; side += 2) {
          sol = (side*size[i]-lpnt[i])/lvec[i];
          if (sol >= 0) {
            const double p0 = lpnt[iface[i][0]] + sol*lvec[iface[i][0]];
            const double p1 = lpnt[iface[i][1]] + sol*lvec[iface[i][1]];
            if (fabs(p0) <= size[iface[i][0]] && fabs(p1) <= size[iface[i][1]]) {
              if (x < 0 || sol < x) x = sol;
            }
          }
        }
      }
    }
    return x;
  }
  if (type == mjhipGEOM_CYLINDER && fabs(lvec[2]) > MINVAL) {   // ray_cylinder flat sides
    for (int side = -1; side <= 1; side += 2) {
      sol = (side*size[1]-lpnt[2])/lvec[2];
      if (sol >= 0) {
        const double p0 = lpnt[0] + sol*lvec[0], p1 = lpnt[1] + sol*lvec[1];
        if (p0*p0 + p1*p1 <= size[0]*size[0]) {
          if (x < 0 || sol < x) x = sol;
        }
      }
    }
  }
  // round side between the flat sides (cylinder :360-380, capsule :250-265)
  double a = lvec[0]*lvec[0] + lvec[1]*lvec[1];
  double b = lvec[0]*lpnt[0] + lvec[1]*lpnt[1];
  double c = lpnt[0]*lpnt[0] + lpnt[1]*lpnt[1] - size[0]*size[0];
  sol = rayQuad(a, b, c, xx);
  if (sol >= 0 && fabs(lpnt[2]+sol*lvec[2]) <= size[1]) {
    if (x < 0 || sol < x) x = sol;
  }
  if (type == mjhipGEOM_CAPSULE) {                      // hemispheres :267-300
    double ldif[3] = {lpnt[0], lpnt[1], lpnt[2]-size[1]};
    a = lvec[0]*lvec[0] + lvec[1]*lvec[1] + lvec[2]*lvec[2];
    b = lvec[0]*ldif[0] + lvec[1]*ldif[1] + lvec[2]*ldif[2];
    c = ldif[0]*ldif[0] + ldif[1]*ldif[1] + ldif[2]*ldif[2] - size[0]*size[0];
    rayQuad(a, b, c, xx);
    for (int i = 0; i < 2; i++) {
      if (xx[i] >= 0 && lpnt[2]+xx[i]*lvec[2] >= size[1]) {
        if (x < 0 || xx[i] < x) x = xx[i];
      }
    }
    ldif[2] = lpnt[2]+size[1];
    b = lvec[0]*ldif[0] + lvec[1]*ldif[1] + lvec[2]*ldif[2];
    c = ldif[0]*ldif[0] + ldif[1]*ldif[1] + ldif[2]*ldif[2] - size[0]*size[0];
    rayQuad(a, b, c, xx);
    for (int i = 0; i < 2; i++) {
      if (xx[i] >= 0 && lpnt[2]+xx[i]*lvec[2] <= -size[1]) {
        if (x < 0 || xx[i] < x) x = xx[i];
      }
    }
  }
  return x;
}

// ray_box :387-445 with each face's hit in all (-1 for none)
MJH_HD double rayBoxAll(const double* pos, const double* mat, const double* size,
                        const double* pnt, const double* vec, double all[6]) {
  for (int i = 0; i < 6; i++) all[i] = -1;
  if (raySphere(pos, size[0]*size[0] + size[1]*size[1] + size[2]*size[2], pnt, vec) < 0) {
    return -1;
  }
  const int iface[3][2] = {{1, 2}, {0, 2}, {0, 1}};
  double lpnt[3], lvec[3], x = -1, sol;
  rayMap(pos, mat, pnt, vec, lpnt, lvec);
  for (int i = 0; i < 3; i++) {
    if (fabs(lvec[i]) > MINVAL) {
      for (int side = -1; side <= 1; side += 2) {
        sol = (side*size[i]-lpnt[i])/lvec[i];
        if (sol >= 0) {
          const double p0 = lpnt[iface[i][0]] + sol*lvec[iface[i][0]];
          const double p1 = lpnt[iface[i][1]] + sol*lvec[iface[i][1]];
          if (fabs(p0) <= size[iface[i][0]] && fabs(p1) <= size[iface[i][1]]) {
            if (x < 0 || sol < x) x = sol;
            all[2*i + (side + 1)/2] = sol;
          }
        }
      }
    }
  }
  return x;
}

// ray_triangle :132-186
MJH_HD double rayTriangle(const double v[3][3], const double* lpnt, const double* lvec,
                          const double* b0, const double* b1) {
  double dif[3][3], planar[3][2];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) dif[i][j] = v[i][j] - lpnt[j];
  }
  for (int i = 0; i < 3; i++) {
    planar[i][0] = dot3(b0, dif[i]);
    planar[i][1] = dot3(b1, dif[i]);
  }
  if ((planar[0][0] > 0 && planar[1][0] > 0 && planar[2][0] > 0) ||
      (planar[0][0] < 0 && planar[1][0] < 0 && planar[2][0] < 0) ||
      (planar[0][1] > 0 && planar[1][1] > 0 && planar[2][1] > 0) ||
      (planar[0][1] < 0 && planar[1][1] < 0 && planar[2][1] < 0)) {
    return -1;
  }
  const double A[4] = {planar[0][0]-planar[2][0], planar[1][0]-planar[2][0],
                       planar[0][1]-planar[2][1], planar[1][1]-planar[2][1]};
  const double b[2] = {-planar[2][0], -planar[2][1]};
  const double det = A[0]*A[3] - A[1]*A[2];
  if (fabs(det) < MINVAL) return -1;
  const double t0 = (A[3]*b[0] - A[1]*b[1]) / det;
  const double t1 = (-A[2]*b[0] + A[0]*b[1]) / det;
  if (t0 < 0 || t1 < 0 || t0 + t1 > 1) return -1;
  double e0[3], e1[3], e2[3], nrm[3];
  sub3(e0, v[0], v[2]);
  sub3(e1, v[1], v[2]);
  sub3(e2, lpnt, v[2]);
  cross(nrm, e0, e1);
  const double denom = dot3(lvec, nrm);
  if (fabs(denom) < MINVAL) return -1;
  return -dot3(e2, nrm) / denom;
}

// the basis of the plane normal to the local ray (mj_rayHfield :497-509, mju_rayTree :651-663)
MJH_HD void rayBasis(const double lvec[3], double b0[3], double b1[3]) {
  b0[0] = b0[1] = b0[2] = 1;
  if (fabs(lvec[0]) >= fabs(lvec[1]) && fabs(lvec[0]) >= fabs(lvec[2])) {
    b0[0] = 0;
  } else if (fabs(lvec[1]) >= fabs(lvec[2])) {
    b0[1] = 0;
  } else {
    b0[2] = 0;
  }
  const double s = -dot3(lvec, b0)/dot3(lvec, lvec);
  for (int k = 0; k < 3; k++) b1[k] = b0[k] + lvec[k]*s;          // mju_addScl3
  normalize3(b1);
  cross(b0, b1, lvec);
  normalize3(b0);
}

// mj_rayHfield :453-595 (the reference's side-face indexing by nrow kept)
MJH_HD double rayHfield(const mjhipModel& m, int id, const double xpos[3], const double xmat[9],
                        const double* pnt, const double* vec) {
  const int hid = m.geom_dataid[id];
  const int nrow = m.hfield_nrow[hid], ncol = m.hfield_ncol[hid];
  const double* size = m.hfield_size + 4*hid;
  const float* data = m.hfield_data + m.hfield_adr[hid];
  const double base_size[3] = {size[0], size[1], size[3]*0.5};
  const double base_pos[3] = {xpos[0] - xmat[2]*size[3]*0.5, xpos[1] - xmat[5]*size[3]*0.5,
                              xpos[2] - xmat[8]*size[3]*0.5};
  const double top_size[3] = {size[0], size[1], size[2]*0.5};
  const double top_pos[3] = {xpos[0] + xmat[2]*size[2]*0.5, xpos[1] + xmat[5]*size[2]*0.5,
                             xpos[2] + xmat[8]*size[2]*0.5};
  double all[6];
  double x = rayBoxAll(base_pos, xmat, base_size, pnt, vec, all);
  const double top_intersect = rayBoxAll(top_pos, xmat, top_size, pnt, vec, all);
  if (top_intersect < 0) return x;
  double lpnt[3], lvec[3], b0[3], b1[3];
  rayMap(xpos, xmat, pnt, vec, lpnt, lvec);
  rayBasis(lvec, b0, b1);
  double seg[2] = {0, top_intersect};
  for (int i = 0; i < 6; i++) {
    if (all[i] > seg[1]) {
      seg[0] = top_intersect;
      seg[1] = all[i];
    }
  }
  const double dx = (2.0*size[0]) / (ncol-1), dy = (2.0*size[1]) / (nrow-1);
  double SX[2], SY[2];
  for (int i = 0; i < 2; i++) {
    SX[i] = (lpnt[0] + seg[i]*lvec[0] + size[0]) / dx;
    SY[i] = (lpnt[1] + seg[i]*lvec[1] + size[1]) / dy;
  }
  int cmin = (int)floor(SX[0] < SX[1] ? SX[0] : SX[1]) - 1;
  int cmax = (int)ceil(SX[0] > SX[1] ? SX[0] : SX[1]) + 1;
  int rmin = (int)floor(SY[0] < SY[1] ? SY[0] : SY[1]) - 1;
  int rmax = (int)ceil(SY[0] > SY[1] ? SY[0] : SY[1]) + 1;
  cmin = cmin > 0 ? cmin : 0;
  cmax = cmax < ncol-1 ? cmax : ncol-1;
  rmin = rmin > 0 ? rmin : 0;
  rmax = rmax < nrow-1 ? rmax : nrow-1;
  for (int r = rmin; r < rmax; r++) {
    for (int c = cmin; c < cmax; c++) {
      const double va[3][3] = {
        {dx*c-size[0], dy*r-size[1], data[r*ncol+c]*size[2]},
        {dx*(c+1)-size[0], dy*(r+1)-size[1], data[(r+1)*ncol+(c+1)]*size[2]},
        {dx*(c+1)-size[0], dy*r-size[1], data[r*ncol+(c+1)]*size[2]}};
      double sol = rayTriangle(va, lpnt, lvec, b0, b1);
      if (sol >= 0 && (x < 0 || sol < x)) x = sol;
      const double vb[3][3] = {
        {dx*c-size[0], dy*r-size[1], data[r*ncol+c]*size[2]},
        {dx*(c+1)-size[0], dy*(r+1)-size[1], data[(r+1)*ncol+(c+1)]*size[2]},
        {dx*c-size[0], dy*(r+1)-size[1], data[(r+1)*ncol+c]*size[2]}};
      sol = rayTriangle(vb, lpnt, lvec, b0, b1);
      if (sol >= 0 && (x < 0 || sol < x)) x = sol;
    }
  }
  for (int i = 0; i < 4; i++) {
    if (all[i] >= 0 && (all[i] < x || x < 0)) {
      const double z = (lpnt[2] + all[i]*lvec[2]) / size[2];
      double y, y0, z0, z1;
      if (i < 2) {
        y = (lpnt[1] + all[i]*lvec[1] + size[1]) / dy;
        y0 = floor(y) < nrow-2 ? floor(y) : nrow-2;
        y0 = y0 > 0 ? y0 : 0;
        z0 = (double)data[(int)round(y0)*nrow + (i == 1 ? ncol-1 : 0)];
        z1 = (double)data[(int)round(y0+1)*nrow + (i == 1 ? ncol-1 : 0)];
      } else {
        y = (lpnt[0] + all[i]*lvec[0] + size[0]) / dx;
        y0 = floor(y) < ncol-2 ? floor(y) : ncol-2;
        y0 = y0 > 0 ? y0 : 0;
        z0 = (double)data[(int)round(y0) + (i == 3 ? (nrow-1)*ncol : 0)];
        z1 = (double)data[(int)round(y0+1) + (i == 3 ? (nrow-1)*ncol : 0)];
      }
      if (z < z0*(y0+1-y) + z1*(y-y0)) x = all[i];
    }
  }
  return x;
}

// mj_rayMesh :800-813: the bounding box, then every face (mju_rayTree :628-730 visits the
// faces whose bounding volumes the ray crosses; the nearest hit over all faces is the same)
MJH_HD double rayMesh(const mjhipModel& m, int id, const double xpos[3], const double xmat[9],
                      const double* pnt, const double* vec) {
  double all[6];
  if (rayBoxAll(xpos, xmat, m.geom_size + 3*id, pnt, vec, all) < 0) return -1;
  const int mid = m.geom_dataid[id];
  double lpnt[3], lvec[3], b0[3], b1[3];
  rayMap(xpos, xmat, pnt, vec, lpnt, lvec);
  rayBasis(lvec, b0, b1);
  double x = -1;
  for (int f = m.mesh_faceadr[mid]; f < m.mesh_faceadr[mid] + m.mesh_facenum[mid]; f++) {
    double v[3][3];
    for (int i = 0; i < 3; i++) {
      const float* vf = m.mesh_vert + 3*(m.mesh_face[3*f + i] + m.mesh_vertadr[mid]);
      for (int j = 0; j < 3; j++) v[i][j] = (double)vf[j];
    }
    const double sol = rayTriangle(v, lpnt, lvec, b0, b1);
    if (sol >= 0 && (x < 0 || sol < x)) x = sol;
  }
  return x;
}

// the rangefinder (engine_sensor.c mjSENS_RANGEFINDER): mj_ray from the site along its z
// axis, geomgroup NULL, flg_static 1, the site's body excluded
// :69-100 ray_eliminate (geomgroup NULL, flg_static 1): the excluded body and invisible geoms
MJH_HD bool rayEliminate(const mjhipModel& m, int g, int bodyexclude) {
  if (m.geom_bodyid[g] == bodyexclude) return true;
  const int mat = m.geom_matid[g];
  if (mat < 0) return m.geom_rgba[4*g+3] == 0;
  return m.mat_rgba[4*mat+3] == 0;
}

// :1145-1185 mj_ray (geomgroup NULL, flg_static 1): the nearest hit distance, -1 for none
// (mju_rayGeom is the touch sensor's rayGeom; the mirror's frames go through registers)
template <int S>
MJH_HD double ray(const mjhipModel& m, const Lane<S>& d, const double pnt[3],
                  const double vec[3], int bodyexclude) {
  double dist = -1;
  for (int g = 0; g < m.ngeom; g++) {
    if (rayEliminate(m, g, bodyexclude)) continue;
    double pos[3], mat[9];
    for (int k = 0; k < 3; k++) pos[k] = d.geom_xpos[3*g+k];
    for (int k = 0; k < 9; k++) mat[k] = d.geom_xmat[9*g+k];
    const int t = m.geom_type[g];
    const double nd = t == mjhipGEOM_MESH ? rayMesh(m, g, pos, mat, pnt, vec) :
                      t == mjhipGEOM_HFIELD ? rayHfield(m, g, pos, mat, pnt, vec) :
                      rayGeom(pos, mat, m.geom_size + 3*g, pnt, vec, t);
    if (nd >= 0 && (nd < dist || dist < 0)) dist = nd;
  }
  return dist;
}


// the touch sensor (engine_sensor.c:750-793): the normal forces of the site body's contacts
// whose normal ray from the contact point hits the site's zone
template <int S>
MJH_HD double touchSensor(const mjhipModel& m, const Lane<S>& d, int objid) {
  const int bodyid = m.site_bodyid[objid];
  const int ncon = d.con_cap ? d.con_count[0] : 0;
  double pos[3], mat[9], total = 0;
  for (int k = 0; k < 3; k++) pos[k] = d.site_xpos[3*objid + k];
  for (int k = 0; k < 9; k++) mat[k] = d.site_xmat[9*objid + k];
  for (int j = 0; j < ncon; j++) {
    const int g0 = d.con_geom[2*j], g1 = d.con_geom[2*j + 1];
    const int b0 = g0 >= 0 ? m.geom_bodyid[g0] : -1, b1 = g1 >= 0 ? m.geom_bodyid[g1] : -1;
    const int adr = d.con_efc_address[j];
    if (adr < 0 || (bodyid != b0 && bodyid != b1)) continue;
    double fn;                                         // mj_contactForce, normal component
    const int dim = d.con_dim[j];
    if (m.opt.cone == mjhipCONE_ELLIPTIC || dim == 1) {
      fn = d.efc_force[adr];
    } else {
      fn = 0;
      for (int k = 0; k < 2*(dim-1); k++) fn += d.efc_force[adr + k];
    }
    if (fn <= 0) continue;
    double ray[3], pnt[3];
    for (int k = 0; k < 3; k++) ray[k] = d.con_frame[9*j + k]*fn;
    normalize3(ray);
    if (bodyid == b1) {
      for (int k = 0; k < 3; k++) ray[k] = ray[k]*-1;
    }
    for (int k = 0; k < 3; k++) pnt[k] = d.con_pos[3*j + k];
    if (rayGeom(pos, mat, m.site_size + 3*objid, pnt, ray, m.site_type[objid]) >= 0) {
      total += fn;
    }
  }
  return total;
}

// engine_sensor.c:677-915 mj_sensorAcc
template <int S>
MJH_HD void sensorAcc(const mjhipModel& m, const Lane<S>& d) {
  if (m.opt.disableflags & mjhipDSBL_SENSOR) return;
  bool post = false;
  double tmp[6];
  for (int i = 0; i < m.nsensor; i++) {
    if (m.sensor_needstage[i] != mjhipSTAGE_ACC) continue;
    const int type = m.sensor_type[i], objtype = m.sensor_objtype[i];
    const int objid = m.sensor_objid[i];
    SP<S> out = d.sensordata + m.sensor_adr[i];
    int r;
    if (!post && (type == mjhSENS_ACCELEROMETER || type == mjhSENS_FORCE ||
                  type == mjhSENS_TORQUE || type == mjhSENS_FRAMELINACC ||
                  type == mjhSENS_FRAMEANGACC)) {
      rnePostConstraint(m, d);
      post = true;
    }
    switch (type) {
    case mjhSENS_TOUCH: out[0] = touchSensor(m, d, objid); break;
    case mjhSENS_ACCELEROMETER:
      objectAcceleration(m, d, 6, objid, tmp, 1);
      copy3(out, tmp + 3);
      break;
    case mjhSENS_FORCE:
    case mjhSENS_TORQUE: {
      const int bodyid = m.site_bodyid[objid], rootid = m.body_rootid[bodyid];
      transformSpatial(tmp, d.cfrc_int + 6*bodyid, 1, d.site_xpos + 3*objid,
                       d.subtree_com + 3*rootid, d.site_xmat + 9*objid, true);
      copy3(out, type == mjhSENS_FORCE ? tmp + 3 : tmp);
      break;
    }
    case mjhSENS_ACTUATORFRC: out[0] = d.actuator_force[objid]; break;
    case mjhSENS_JOINTACTFRC: out[0] = d.qfrc_actuator[m.jnt_dofadr[objid]]; break;
    case mjhSENS_JOINTLIMITFRC:
    case mjhSENS_TENDONLIMITFRC:
      out[0] = 0;
      r = limitRow(d, type == mjhSENS_JOINTLIMITFRC ? CNSTR_LIMIT_JOINT : CNSTR_LIMIT_TENDON,
                   objid);
      if (r >= 0) out[0] = d.efc_force[r];
      break;
    case mjhSENS_FRAMELINACC:
    case mjhSENS_FRAMEANGACC:
      objectAcceleration(m, d, objtype, objid, tmp, 0);
      copy3(out, type == mjhSENS_FRAMELINACC ? tmp + 3 : tmp);
      break;
    default: break;
    }
  }
  applyCutoff(m, d, mjhipSTAGE_ACC);
}

// mju_isBad (engine_util_misc.c:1315-1317): NaN or |x| > mjMAXVAL
MJH_HD bool isBad(double x) { return x != x || x > mjhipMAXVAL || x < -mjhipMAXVAL; }

// mj_checkPos / mj_checkVel / mj_checkAcc (engine_forward.c:53-102) on the inputs a call
// reads, as status bits: the batched analogue of their mjWARN_BADQPOS/QVEL/QACC warnings.
// Nothing is reset (a batch never aborts) and no result changes.
template <int S>
MJH_HD int checkInputs(const mjhipModel& m, const Lane<S>& d, int skipstage) {
  int st = 0;
  if (skipstage < mjhipSTAGE_POS) {
    for (int i = 0; i < m.nq; i++) st |= isBad(d.qpos[i]) ? MJHIP_INST_BADQPOS : 0;
  }
  if (skipstage < mjhipSTAGE_VEL) {
    for (int i = 0; i < m.nv; i++) st |= isBad(d.qvel[i]) ? MJHIP_INST_BADQVEL : 0;
  }
  for (int i = 0; i < m.nv; i++) st |= isBad(d.qacc[i]) ? MJHIP_INST_BADQACC : 0;
  return st;
}

// FUSED (the constraint rows finished at creation, see contactRowsFused) requires
// skipstage = mjSTAGE_NONE, no mjENBL_INVDISCRETE, nbody <= 64 and d.chain set (fusedOk)
template <int S, bool CONTACT = true, bool FUSED = false>
MJH_HD int inverseSkip(const mjhipModel& m, const Lane<S>& d, int skipstage,
                       int skipsensor = 0) {
  int status = checkInputs(m, d, skipstage);
  const bool energy = (m.opt.enableflags & mjhipENBL_ENERGY) != 0;
  const bool sensors = !skipsensor && m.nsensor > 0;
  if (skipstage < mjhipSTAGE_POS) {
    invPosition<S, CONTACT, FUSED>(m, d, &status);
    if (sensors) sensorPos(m, d);
    if (energy) energyPos(m, d);
  }
  MJH_PHASE(6);
  if (skipstage < mjhipSTAGE_VEL) {
    invVelocity<S, FUSED>(m, d);
    if (sensors) sensorVel(m, d);
    if (energy) energyVel(m, d);
  }
  MJH_PHASE(7);
  const bool discrete = !FUSED && (m.opt.enableflags & mjhipENBL_INVDISCRETE) != 0;
  if (discrete) {
    copy(d.qacc_save, d.qacc, m.nv);
    discreteAcc(m, d);
  }
  if constexpr (!FUSED) invConstraint(m, d);
  MJH_PHASE(8);
  rne(m, d, 1, d.qfrc_inverse);
  if (sensors) sensorAcc(m, d);
  for (int i = 0; i < m.nv; i++) {
    d.qfrc_inverse[i] += m.dof_armature[i] * d.qacc[i]
                         - d.qfrc_passive[i] - d.qfrc_constraint[i];
  }
  if (discrete) copy(d.qacc, d.qacc_save, m.nv);
  MJH_PHASE(9);
  return status;
}

// mj_transmission (engine_core_smooth.c:996-1318) of the slider-crank, site and body
// actuators and their actuator_velocity (mj_fwdVelocity, engine_forward.c:214-219) after the
// generated kernels and the constraint part. No other mj_inverse output reads them (the
// inverse forces do not involve actuators), the sensors after this do, and a body
// transmission reads this instance's contacts, which the constraint part made.
template <int S>
MJH_HD void transmissionAfter(const mjhipModel& m, const Lane<S>& d) {
  transmission(m, d, true);
  if (m.opt.disableflags & mjhipDSBL_ACTUATION) return;
  for (int r = 0; r < m.nu; r++) {
    if (!mjh_trnAfter(m.actuator_trntype[r])) continue;
    const int adr = m.moment_rowadr[r];
    d.actuator_velocity[r] = dotSparse(d.actuator_moment + adr, d.qvel, m.moment_rownnz[r],
                                       m.moment_colind + adr);
  }
}

// mj_sensorPos/Vel/Acc and mj_energyPos/Vel of mj_inverseSkip(mjSTAGE_NONE) after the
// generated kernels and the constraint part, in the reference's order: every sensor and
// energy term reads only its own stage's fields, which no later stage rewrites, and none
// reads qfrc_inverse, so running them after the whole pass gives the reference's values
template <int S>
MJH_HD void sensorsAfter(const mjhipModel& m, const Lane<S>& d, bool sensors = true,
                         bool trn = false) {
  if (trn) transmissionAfter(m, d);
  sensors = sensors && m.nsensor > 0;
  const bool energy = (m.opt.enableflags & mjhipENBL_ENERGY) != 0;
  if (sensors) sensorPos(m, d);
  if (energy) energyPos(m, d);
  if (sensors) sensorVel(m, d);
  if (energy) energyVel(m, d);
  if (sensors) sensorAcc(m, d);
}

// The constraint part of mj_inverseSkip(mjSTAGE_NONE) for an instance whose constraint-free
// stages the generated kernels (codegen.py) already wrote to the mirror, with the raw
// mj_rne(flg_acc = 1) result left in qfrc_inverse: collision, mj_makeConstraint and its
// velocity/acceleration-stage parts, then the reference's assembly
// qfrc_inverse = rne + ((armature*qacc - qfrc_passive) - qfrc_constraint).
template <int S, bool CONTACT, bool FUSED>
MJH_HD int constraintOnly(const mjhipModel& m, const Lane<S>& d) {
  int status = 0;
  MJH_PHASE0(10, 25);
  if constexpr (CONTACT) collision(m, d, &status);
  else d.con_count[0] = 0;
  MJH_PHASE(11);
  makeConstraint<S, CONTACT, FUSED>(m, d, &status);
  MJH_PHASE(12);
  if constexpr (!FUSED) {
    referenceConstraint(m, d);
    invConstraint(m, d);
  }
  MJH_PHASE(13);
  for (int i = 0; i < m.nv; i++) {
    d.qfrc_inverse[i] += m.dof_armature[i] * d.qacc[i]
                         - d.qfrc_passive[i] - d.qfrc_constraint[i];
  }
  return status;
}

//---------------------------------- engine_forward.c (constraint-free) ----------------------

// mj_fwdActuation :276-515 for joint transmissions with fixed/affine gain and none/affine
// bias (the actuator subset accepted at context creation); ctrl clamped by ctrlrange
template <int S>
MJH_HD void fwdActuation(const mjhipModel& m, const Lane<S>& d) {
  const int nv = m.nv, nu = m.nu;
  zero(d.qfrc_actuator, nv);
  zero(d.actuator_force, nu);
  if ((m.opt.disableflags & mjhipDSBL_ACTUATION) || !nu) return;
  for (int i = 0; i < nu; i++) {
    double ctrl = d.ctrl[i];
    if (m.actuator_ctrllimited[i] && !(m.opt.disableflags & mjhipDSBL_CLAMPCTRL)) {
      const double* r = m.actuator_ctrlrange + 2*i;
      ctrl = ctrl < r[0] ? r[0] : (ctrl > r[1] ? r[1] : ctrl);
    }
    const double* prm = m.actuator_gainprm + 10*i;
    double gain = prm[0];
    if (m.actuator_gaintype[i] == mjhipGAIN_AFFINE) {
      gain = prm[0] + prm[1]*d.actuator_length[i] + prm[2]*d.actuator_velocity[i];
    }
    double f = gain * ctrl;
    if (m.actuator_biastype[i] == mjhipBIAS_AFFINE) {
      prm = m.actuator_biasprm + 10*i;
      f += prm[0] + prm[1]*d.actuator_length[i] + prm[2]*d.actuator_velocity[i];
    }
    if (m.actuator_forcelimited[i]) {
      const double* r = m.actuator_forcerange + 2*i;
      f = f < r[0] ? r[0] : (f > r[1] ? r[1] : f);
    }
    d.actuator_force[i] = f;
  }
  for (int i = 0; i < nu; i++) {            // mju_mulMatTVecSparse
    double f = d.actuator_force[i];
    if (!f) continue;
    int adr = m.moment_rowadr[i];
    for (int j = 0; j < m.moment_rownnz[i]; j++) {
      d.qfrc_actuator[m.moment_colind[adr+j]] += d.actuator_moment[adr+j]*f;
    }
  }
}

// mj_xfrcAccumulate engine_support.c:1254-1261
template <int S>
MJH_HD void xfrcAccumulate(const mjhipModel& m, const Lane<S>& d, SP<S> qfrc) {
  for (int i = 1; i < m.nbody; i++) {
    SP<S> x = d.xfrc_applied + 6*i;
    if (x[0] || x[1] || x[2] || x[3] || x[4] || x[5]) {
      applyFT(m, d, x, x + 3, d.xipos + 3*i, i, qfrc);
    }
  }
}

// mj_forward without constraint rows: fwdPosition = invPosition, fwdVelocity, fwdActuation,
// fwdAcceleration (:520-531), then mj_fwdConstraint with nefc = 0: qacc = qacc_smooth.
// Instances with constraint rows (the constraint solver is not implemented) are flagged
// MJHIP_INST_UNSUPPORTED and get qacc = qacc_smooth.
template <int S, bool CONTACT = true>
MJH_HD int forwardSkip(const mjhipModel& m, const Lane<S>& d, int skipstage) {
  const int nv = m.nv;
  int status = 0;
  for (int i = 0; i < m.nq; i++) status |= isBad(d.qpos[i]) ? MJHIP_INST_BADQPOS : 0;
  for (int i = 0; i < nv; i++) status |= isBad(d.qvel[i]) ? MJHIP_INST_BADQVEL : 0;
  if (skipstage < mjhipSTAGE_POS) invPosition<S, CONTACT>(m, d, &status);
  if (skipstage < mjhipSTAGE_VEL) invVelocity(m, d);
  fwdActuation(m, d);
  for (int i = 0; i < nv; i++) d.qfrc_smooth[i] = d.qfrc_passive[i] - d.qfrc_bias[i];
  addTo(d.qfrc_smooth, d.qfrc_applied, nv);
  addTo(d.qfrc_smooth, d.qfrc_actuator, nv);
  xfrcAccumulate(m, d, d.qfrc_smooth);
  copy(d.qacc_smooth, d.qfrc_smooth, nv);
  solveM(m, d, d.qacc_smooth);
  copy(d.qacc, d.qacc_smooth, nv);
  zero(d.qfrc_constraint, nv);
  for (int i = 0; i < nv; i++) status |= isBad(d.qacc[i]) ? MJHIP_INST_BADQACC : 0;
  if (d.efc_count[0] > 0) status |= MJHIP_INST_UNSUPPORTED;
  return status;
}

}  // namespace mjh

//---------------------------------- device mirror (include/mjhip.h layout) ------------------

struct Mirror {
#define XD(name, d0, d1, stage) double* name; int name##_n;
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
#undef XD
#define XSC(name, n) double* name; int name##_n;
  MJHIP_SCRATCH_FIELDS
#undef XSC
#define XSI(name, n) int* name; int name##_n;
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
  int efc_cap;
  int con_cap;
  long nj_cap;
  const CoopPair* prog;                      // the static collision program (Lane::prog)
  const int* prog_ipair;
  int nprog;
  // mjd_inverseFD's perturbed instances (codegen.FD_KEEP): fd_elide set, the generated
  // kernels' FD instantiation drops, from instance block full_blk on, the stores no later
  // kernel reads
  int fd_elide;
  int full_blk;
};

MJH_HD mjh::Lane<64> lane_view(const Mirror& mr, int blk, int lane) {
  mjh::Lane<64> d;
#define XD(name, d0, d1, stage) d.name.p = mr.name + ((long)blk*mr.name##_n)*64 + lane;
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
#undef XD
#undef XSCC
#undef XSIC
#define XSC(name, n) d.name.p = mr.name + ((long)blk*mr.name##_n)*64 + lane;
#define XSCC(name, n) d.name.p = mr.name + ((long)blk*64 + lane)*mr.name##_n;
  MJHIP_SCRATCH_FIELDS
#undef XSC
#define XSI(name, n) d.name.p = mr.name + ((long)blk*mr.name##_n)*64 + lane;
#define XSIC(name, n) d.name.p = mr.name + ((long)blk*64 + lane)*mr.name##_n;
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
#undef XSCC
#undef XSIC
#define XSCC(name, n) XSC(name, n)
#define XSIC(name, n) XSI(name, n)
  d.efc_cap = mr.efc_cap;
  d.con_cap = mr.con_cap;
  d.nj_cap = mr.nj_cap;
  d.chain = nullptr;
  d.gxpos = d.geom_xpos;
  d.gstage = false;
  d.prog = mr.prog;
  d.prog_ipair = mr.prog_ipair;
  d.nprog = mr.nprog;
  d.cdq = nullptr;
  d.fst = nullptr;
  d.nfst = 0;
  d.cbody = nullptr;
  d.ncbody = 0;
  d.dchain = nullptr;
  d.ccdx = mr.ccd + ((long)blk*mr.ccd_n)*64 + (long)lane*mr.ccd_n;
  d.ccdxi = mr.ccdi + ((long)blk*mr.ccdi_n)*64 + (long)lane*mr.ccdi_n;
  return d;
}

#if defined(__HIPCC__)
  #define MJH_ATOMIC_ADD(p, v) atomicAdd((p), (v))
#else
  #define MJH_ATOMIC_ADD(p, v) ((*(p) += (v)) - (v))
#endif

// Value barrier: the compiler must treat x as recomputed here, so expressions of x after the
// barrier are not merged with the same expressions before it (used by the generated kernels
// to recompute kinematics instead of keeping the first pass's frames live). No code emitted.
#if defined(__HIP_DEVICE_COMPILE__)
  #define MJH_OPAQUE(x) asm volatile("" : "+v"(x))
#else
  #define MJH_OPAQUE(x) asm volatile("" : "+m"(x))
#endif

// Scheduling fence for the generated kernels: the machine scheduler may not move any
// instruction across it. It keeps a body's prefetched loads from being hoisted to the top of
// the kernel, where they would all be live at once and spill.
#if defined(__HIP_DEVICE_COMPILE__)
  #define MJH_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
  #define MJH_SCHED_FENCE() ((void)0)
#endif

// Compiler memory barrier (no instruction): values written to LDS before it are re-read from
// LDS after it instead of being forwarded in registers.
#define MJH_MEM_BARRIER() asm volatile("" ::: "memory")

// sin and cos of one argument (device: one shared argument reduction)
#if defined(__HIP_DEVICE_COMPILE__)
  #define MJH_SINCOS(x, s, c) sincos((x), &(s), &(c))
#else
  #define MJH_SINCOS(x, s, c) ((s) = sin(x), (c) = cos(x))
#endif

#endif  // MJHIP_ENGINE_DEVICE_H_
