/* mj_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's inverse-dynamics path (MuJoCo 3.3.1 fork,
 * fancifulland2718/mujoco_InverseDynamicsTest), used as the parity checker for the HIP
 * engine. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so; the product library (libmjhip.so) never links or calls it.
 *
 * Parity pinning: the reference cannot be built in this image (src/engine/engine_support.c
 * includes engine_collision_convex.h -> <ccd/vec3.h>, libccd v2.1 @7931e764 is absent and
 * stand-in headers are not allowed), so this restatement is pinned by the reference's own
 * known-answer/property tests restated in tests/test_oracle_pins.py (LinearSystemInverse,
 * FactorI/FactorIs, SolveLDs, MjDataWorldBodyValuesAreInitialized, the fwd/inv identity of
 * src/inverse/inverse_test.cpp and mj_compareFwdInv) — there are no golden vectors in the
 * reference. Summation orders follow the scalar (non-AVX) reference code, which the
 * reference states reproduces its AVX order for mju_dot (engine_util_blas.c:715-729).
 */
#ifndef MJ_ORACLE_H_
#define MJ_ORACLE_H_

#include "../include/mjhip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* constraint rows (the reference's efc_* arena arrays, mjxmacro.h MJDATA_ARENA_POINTERS) */
typedef struct orEfc_ {
  int capacity;       /* rows allocated */
  int nefc, ne, nf, nl;
  int* efc_type;      /* mjtConstraint */
  int* efc_id;
  int* efc_state;     /* mjtConstraintState */
  mjtNum* efc_J;      /* capacity x nv: dense rows, or compressed rows (sparse mode) */
  mjtNum* efc_pos;
  mjtNum* efc_margin;
  mjtNum* efc_frictionloss;
  mjtNum* efc_diagApprox;
  mjtNum* efc_KBIP;   /* capacity x 4 */
  mjtNum* efc_D;
  mjtNum* efc_R;
  mjtNum* efc_vel;
  mjtNum* efc_aref;
  mjtNum* efc_force;
  /* contacts (the mjContact fields this path uses), SoA over con_capacity entries */
  int con_capacity;
  int ncon;
  mjtNum* con_dist;
  mjtNum* con_pos;             /* x3 */
  mjtNum* con_frame;           /* x9 */
  mjtNum* con_includemargin;
  mjtNum* con_friction;        /* x5 */
  mjtNum* con_solref;          /* x2 */
  mjtNum* con_solreffriction;  /* x2 */
  mjtNum* con_solimp;          /* x5 */
  mjtNum* con_mu;
  int* con_dim;
  int* con_geom;               /* x2 */
  int* con_exclude;
  int* con_efc_address;
  /* sparse-mode models (mj_isSparse): efc_J holds compressed rows (capacity x nv doubles of
   * room), described by these arrays, and efc_JT their transpose (mj_makeConstraint
   * engine_core_constraint.c:2083-2104) */
  int nJ;
  int* efc_J_rownnz;           /* capacity */
  int* efc_J_rowadr;           /* capacity */
  int* efc_J_colind;           /* capacity x nv */
  mjtNum* efc_JT;              /* capacity x nv */
  int* efc_JT_rownnz;          /* nv */
  int* efc_JT_rowadr;          /* nv */
  int* efc_JT_colind;          /* capacity x nv */
} orEfc;

/* mjtConstraint / mjtConstraintState values (mjmodel.h) */
enum { orCNSTR_EQUALITY = 0, orCNSTR_FRICTION_DOF, orCNSTR_FRICTION_TENDON,
       orCNSTR_LIMIT_JOINT, orCNSTR_LIMIT_TENDON, orCNSTR_CONTACT_FRICTIONLESS,
       orCNSTR_CONTACT_PYRAMIDAL, orCNSTR_CONTACT_ELLIPTIC };
enum { orCNSTRSTATE_SATISFIED = 0, orCNSTRSTATE_QUADRATIC, orCNSTRSTATE_LINEARNEG,
       orCNSTRSTATE_LINEARPOS, orCNSTRSTATE_CONE };

int  or_efcCapacity(const mjhipModel* m);
/* mjd_smooth_vel on the D sparsity (D_rowadr/D_colind), from the fields already in d */
void or_smoothVel(const mjhipModel* m, const mjhipData* d, mjtNum* qDeriv, int flg_bias);
int  or_contactCapacity(const mjhipModel* m);   /* -1: unsupported collision pair */

/* pipeline (engine_inverse.c) */
void or_inverseSkip(const mjhipModel* m, mjhipData* d, orEfc* efc, int skipstage,
                    int skipsensor);
void or_inverse(const mjhipModel* m, mjhipData* d, orEfc* efc);

/* the stage functions of mj_inverseSkip (engine_inverse.c:37-68, :73-76, :169-192) */
void or_invPosition(const mjhipModel* m, mjhipData* d, orEfc* efc);
void or_invVelocity(const mjhipModel* m, mjhipData* d, orEfc* efc);
void or_invConstraint(const mjhipModel* m, mjhipData* d, orEfc* efc);

/* individual stages, exported for the pin tests */
void or_kinematics(const mjhipModel* m, mjhipData* d);
void or_comPos(const mjhipModel* m, mjhipData* d);
void or_crb(const mjhipModel* m, mjhipData* d);
void or_factorM(const mjhipModel* m, mjhipData* d);
void or_solveM(const mjhipModel* m, const mjhipData* d, mjtNum* x, const mjtNum* y, int n);
void or_rne(const mjhipModel* m, mjhipData* d, int flg_acc, mjtNum* result);
void or_fullM(const mjhipModel* m, mjtNum* dst, const mjtNum* M);

/* forward dynamics harness for the fwd/inv identity (engine_forward.c), constraint-free
 * states only: returns nefc (the caller checks 0) */
int  or_forward(const mjhipModel* m, mjhipData* d, orEfc* efc);
void or_xfrcAccumulate(const mjhipModel* m, mjhipData* d, mjtNum* qfrc);
void or_rungeKutta4(const mjhipModel* m, mjhipData* d, orEfc* efc);

/* mjd_inverseFD (engine_derivative_fd.c:611-719), flg_actuation = 0; any output may be NULL,
 * sensors are skipped when DsDq, DsDv and DsDa are all NULL */
void or_inverseFD(const mjhipModel* m, mjhipData* d, orEfc* efc, mjtNum eps,
                  mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa, mjtNum* DsDq, mjtNum* DsDv,
                  mjtNum* DsDa, mjtNum* DmDq);
/* the same with the reference's flg_actuation (force = qfrc_inverse - qfrc_actuator of
 * mj_fwdActuation, engine_derivative_fd.c:160-168; d->ctrl is the control) */
void or_inverseFDEx(const mjhipModel* m, mjhipData* d, orEfc* efc, mjtNum eps,
                    int flg_actuation, mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa, mjtNum* DsDq,
                    mjtNum* DsDv, mjtNum* DsDa, mjtNum* DmDq);

/* test hooks: the reference tests' Penetration helper (mjc_ccd, one contact; returns the
 * count, out = dist, dir[3], pos[3]) and mj_ray (geomgroup NULL, flg_static 1) */
int or_ccdPenetration(const mjhipModel* m, const mjhipData* d, int g1, int g2, mjtNum margin,
                      mjtNum tol, int kmax, mjtNum* out);
mjtNum or_ccdGeneral(const mjhipModel* m, const mjhipData* d, int g1, int g2, mjtNum margin,
                     mjtNum tol, int kmax, int maxc, mjtNum cutoff, mjtNum* out);
mjtNum or_rayTest(const mjhipModel* m, const mjhipData* d, const mjtNum* pnt,
                  const mjtNum* vec, int bodyexclude, int* geomid);

/* mj_compareFwdInv (engine_inverse.c:275-316) on the rows in efc (a forward pass's) */
void or_compareFwdInv(const mjhipModel* m, mjhipData* d, orEfc* efc);

/* CPU baseline: B instances of mj_inverse over `nthread` threads, one data per thread,
 * static chunks of B/(10*nthread) (python/mujoco/rollout.cc:307-317). Returns seconds. */
double or_inverseBatch(const mjhipModel* m, int B, const mjtNum* qpos, const mjtNum* qvel,
                       const mjtNum* qacc, mjtNum* qfrc_inverse, int nthread);

#ifdef __cplusplus
}
#endif

#endif  /* MJ_ORACLE_H_ */
