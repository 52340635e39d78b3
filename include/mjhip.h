/* mjhip.h — C-ABI of the MI355X batched inverse-dynamics engine (libmjhip.so).
 *
 * This is the drop-in boundary for the reference's inverse-dynamics path
 * (fancifulland2718/mujoco_InverseDynamicsTest = MuJoCo 3.3.1 + local edits):
 *
 *   reference entry point (file:line)                          replaced by
 *   ---------------------------------------------------------  -------------------------------
 *   mj_inverse        src/engine/engine_inverse.c:266          mjhip_inverse
 *                     include/mujoco/mujoco.h:131
 *   mj_inverseSkip    src/engine/engine_inverse.c:197          mjhip_inverseSkip
 *                     include/mujoco/mujoco.h:137
 *   mj_invPosition    src/engine/engine_inverse.c:37           mjhip_invPosition
 *                     src/engine/engine_inverse.h:34
 *   mj_invVelocity    src/engine/engine_inverse.c:73           mjhip_invVelocity
 *                     src/engine/engine_inverse.h:37
 *   mj_invConstraint  src/engine/engine_inverse.c:169          mjhip_invConstraint
 *                     src/engine/engine_inverse.h:40
 *   mj_compareFwdInv  src/engine/engine_inverse.c:275          mjhip_compareFwdInv
 *                     src/engine/engine_inverse.h:43
 *   mj_rne            src/engine/engine_core_smooth.c:1969     mjhip_rne
 *                     include/mujoco/mujoco.h:361
 *   mjd_inverseFD     src/engine/engine_derivative_fd.c:611    mjhip_inverseFDBatch (batched)
 *                     include/mujoco/mujoco.h:1244-1247
 *   (batch of mj_inverse calls over one mjModel, the data-parallel pattern of
 *    python/mujoco/rollout.cc:180-220 and sample/testspeed.cc:177-227)
 *                                                              mjhip_inverseBatch
 *
 * Types: mjtNum is double (include/mujoco/mjtnum.h:21-22); mjtByte is unsigned char.
 * mjhipModel / mjhipData hold the reference's field names, element types and row-major
 * shapes (include/mujoco/mjxmacro.h), so a maintainer's adapter can fill them by plain
 * pointer assignment from a real mjModel/mjData.
 *
 * Errors: the reference has no return codes (fatal -> mju_error, soft -> mj_warning,
 * engine_util_errmem.c:118-150, engine_support.c:1650-1667). The single-instance entry
 * points keep that behaviour through a user-settable error callback; the batch entry
 * points return an mjhipStatus and never exit. Every compute entry point runs on the GPU;
 * there is no CPU fallback: without a usable HIP device the call fails with
 * MJHIP_ERR_NO_DEVICE.
 */
#ifndef MJHIP_H_
#define MJHIP_H_

#include <stddef.h>
#include <stdint.h>

#include "mjhip_fields.h"

#ifdef __cplusplus
extern "C" {
#endif

#if defined(_WIN32)
  #define MJHIP_API __declspec(dllexport)
#else
  #define MJHIP_API __attribute__((visibility("default")))
#endif

typedef double mjtNum;
typedef unsigned char mjtByte;

/*---------------------------- constants (include/mujoco/mjmodel.h:24-45, mjtnum.h:23) ----*/
#define mjhipPI      3.14159265358979323846
#define mjhipMINVAL  1E-15
#define mjhipMAXVAL  1E+10
#define mjhipMINIMP  0.0001
#define mjhipMAXIMP  0.9999
#define mjhipNREF    2
#define mjhipNIMP    5
#define mjhipNEQDATA 11

/*---------------------------- enums: same values as the reference ------------------------*/
typedef enum mjhipDisableBit_ {      /* mjmodel.h:50-68 */
  mjhipDSBL_CONSTRAINT   = 1 << 0,
  mjhipDSBL_EQUALITY     = 1 << 1,
  mjhipDSBL_FRICTIONLOSS = 1 << 2,
  mjhipDSBL_LIMIT        = 1 << 3,
  mjhipDSBL_CONTACT      = 1 << 4,
  mjhipDSBL_PASSIVE      = 1 << 5,
  mjhipDSBL_GRAVITY      = 1 << 6,
  mjhipDSBL_CLAMPCTRL    = 1 << 7,
  mjhipDSBL_WARMSTART    = 1 << 8,
  mjhipDSBL_FILTERPARENT = 1 << 9,
  mjhipDSBL_ACTUATION    = 1 << 10,
  mjhipDSBL_REFSAFE      = 1 << 11,
  mjhipDSBL_SENSOR       = 1 << 12,
  mjhipDSBL_MIDPHASE     = 1 << 13,
  mjhipDSBL_EULERDAMP    = 1 << 14,
  mjhipDSBL_AUTORESET    = 1 << 15,
  mjhipDSBL_NATIVECCD    = 1 << 16
} mjhipDisableBit;

typedef enum mjhipEnableBit_ {       /* mjmodel.h:70-79 */
  mjhipENBL_OVERRIDE    = 1 << 0,
  mjhipENBL_ENERGY      = 1 << 1,
  mjhipENBL_FWDINV      = 1 << 2,
  mjhipENBL_INVDISCRETE = 1 << 3,
  mjhipENBL_MULTICCD    = 1 << 4,
  mjhipENBL_ISLAND      = 1 << 5
} mjhipEnableBit;

typedef enum mjhipJoint_ {           /* mjmodel.h mjtJoint */
  mjhipJNT_FREE = 0, mjhipJNT_BALL, mjhipJNT_SLIDE, mjhipJNT_HINGE
} mjhipJoint;

typedef enum mjhipGeom_ {            /* mjmodel.h mjtGeom */
  mjhipGEOM_PLANE = 0, mjhipGEOM_HFIELD, mjhipGEOM_SPHERE, mjhipGEOM_CAPSULE,
  mjhipGEOM_ELLIPSOID, mjhipGEOM_CYLINDER, mjhipGEOM_BOX, mjhipGEOM_MESH, mjhipGEOM_SDF
} mjhipGeom;

typedef enum mjhipCamLight_ {        /* mjmodel.h mjtCamLight */
  mjhipCAMLIGHT_FIXED = 0, mjhipCAMLIGHT_TRACK, mjhipCAMLIGHT_TRACKCOM,
  mjhipCAMLIGHT_TARGETBODY, mjhipCAMLIGHT_TARGETBODYCOM
} mjhipCamLight;

typedef enum mjhipEq_ {              /* mjmodel.h mjtEq */
  mjhipEQ_CONNECT = 0, mjhipEQ_WELD, mjhipEQ_JOINT, mjhipEQ_TENDON, mjhipEQ_FLEX,
  mjhipEQ_DISTANCE
} mjhipEq;

typedef enum mjhipWrap_ {            /* mjmodel.h:191-198 */
  mjhipWRAP_NONE = 0, mjhipWRAP_JOINT, mjhipWRAP_PULLEY, mjhipWRAP_SITE,
  mjhipWRAP_SPHERE, mjhipWRAP_CYLINDER
} mjhipWrap;

typedef enum mjhipTrn_ {             /* mjmodel.h:201-210 */
  mjhipTRN_JOINT = 0, mjhipTRN_JOINTINPARENT, mjhipTRN_SLIDERCRANK, mjhipTRN_TENDON,
  mjhipTRN_SITE, mjhipTRN_BODY, mjhipTRN_UNDEFINED = 1000
} mjhipTrn;

typedef enum mjhipDyn_ {             /* mjmodel.h mjtDyn */
  mjhipDYN_NONE = 0, mjhipDYN_INTEGRATOR, mjhipDYN_FILTER, mjhipDYN_FILTEREXACT,
  mjhipDYN_MUSCLE, mjhipDYN_USER
} mjhipDyn;

typedef enum mjhipGain_ {            /* mjmodel.h mjtGain */
  mjhipGAIN_FIXED = 0, mjhipGAIN_AFFINE, mjhipGAIN_MUSCLE, mjhipGAIN_USER
} mjhipGain;

typedef enum mjhipBias_ {            /* mjmodel.h mjtBias */
  mjhipBIAS_NONE = 0, mjhipBIAS_AFFINE, mjhipBIAS_MUSCLE, mjhipBIAS_USER
} mjhipBias;

typedef enum mjhipSameFrame_ {       /* mjmodel.h:379-385 */
  mjhipSAMEFRAME_NONE = 0, mjhipSAMEFRAME_BODY, mjhipSAMEFRAME_INERTIA,
  mjhipSAMEFRAME_BODYROT, mjhipSAMEFRAME_INERTIAROT
} mjhipSameFrame;

typedef enum mjhipStage_ {           /* mjmodel.h:363-368 */
  mjhipSTAGE_NONE = 0, mjhipSTAGE_POS, mjhipSTAGE_VEL, mjhipSTAGE_ACC
} mjhipStage;

typedef enum mjhipIntegrator_ {      /* mjmodel.h mjtIntegrator */
  mjhipINT_EULER = 0, mjhipINT_RK4, mjhipINT_IMPLICIT, mjhipINT_IMPLICITFAST
} mjhipIntegrator;

typedef enum mjhipJacobian_ {        /* mjmodel.h mjtJacobian */
  mjhipJAC_DENSE = 0, mjhipJAC_SPARSE, mjhipJAC_AUTO
} mjhipJacobian;

typedef enum mjhipCone_ {            /* mjmodel.h mjtCone */
  mjhipCONE_PYRAMIDAL = 0, mjhipCONE_ELLIPTIC
} mjhipCone;

/*---------------------------- option (include/mujoco/mjmodel.h mjOption) -----------------*/
typedef struct mjhipOption_ {
  mjtNum timestep;
  mjtNum impratio;
  mjtNum gravity[3];
  mjtNum wind[3];
  mjtNum magnetic[3];        /* magnetometer sensor field (mjmodel.h mjOption) */
  mjtNum density;
  mjtNum viscosity;
  mjtNum o_margin;
  mjtNum o_solref[mjhipNREF];
  mjtNum o_solimp[mjhipNIMP];
  mjtNum o_friction[5];
  mjtNum ccd_tolerance;      /* convex collision solver tolerance (mjOption ccd_tolerance) */
  int integrator;
  int cone;
  int jacobian;
  int disableflags;
  int enableflags;
  int ccd_iterations;        /* convex collision solver iterations (mjOption ccd_iterations) */
} mjhipOption;

/*---------------------------- model: sizes + field pointers ------------------------------*/
typedef struct mjhipModel_ {
#define XS(name) int name;
  MJHIP_MODEL_SIZES
#undef XS
  mjhipOption opt;
#define X(type, name, d0, d1) type* name;
  MJHIP_MODEL_POINTERS
#undef X
} mjhipModel;

/*---------------------------- data (single instance, host memory) ------------------------*/
/* Status bits set per instance by every compute entry point (the batched analogue of the
 * reference's mj_warning counters, engine_support.c:1650-1667, and of the efc overflow
 * warning mjWARN_CNSTRFULL, engine_core_constraint.c:65-72). Nothing aborts a batch. */
typedef enum mjhipInstanceStatus_ {
  MJHIP_INST_OK            = 0,
  MJHIP_INST_BADQPOS       = 1 << 0,   /* nan/|x|>mjMAXVAL in qpos (mj_checkPos semantics) */
  MJHIP_INST_BADQVEL       = 1 << 1,
  MJHIP_INST_BADQACC       = 1 << 2,
  MJHIP_INST_INERTIA       = 1 << 3,   /* small/negative pivot in LTDL (mjWARN_INERTIA) */
  MJHIP_INST_CNSTRFULL     = 1 << 4,   /* more constraint rows than the per-instance capacity */
  MJHIP_INST_UNSUPPORTED   = 1 << 5    /* model feature not implemented on the device path */
} mjhipInstanceStatus;

typedef struct mjhipData_ {
  int nefc;                 /* number of constraint rows of the last call */
  int status;               /* mjhipInstanceStatus bits of the last call */
  mjtNum solver_fwdinv[2];  /* mjdata.h:186, written by mjhip_compareFwdInv */
  mjtNum energy[2];         /* potential, kinetic (mjdata.h energy): written under
                               mjENBL_ENERGY by the stages that run (engine_inverse.c:207-223) */
  mjtNum time;              /* simulation time (mjdata.h time): read by clock sensors */
  /* inputs and every fp64 output field of mj_inverseSkip, reference names */
#define XD(name, d0, d1, stage) mjtNum* name;
  MJHIP_DATA_FIELDS
#undef XD
  /* forward-dynamics inputs/outputs, also read by the fwd/inv comparison harness
   * (inverse_test.cpp:51-73): ctrl, qfrc_applied, xfrc_applied, actuator_force,
   * qfrc_actuator, qfrc_smooth, qacc_smooth */
#define XD(name, d0, d1, stage) mjtNum* name;
  MJHIP_DATA_FORWARD
#undef XD
  /* computed by the sensor stages when a sensor needs them (engine_sensor.c) */
#define XD(name, d0, d1, stage) mjtNum* name;
  MJHIP_DATA_SENSOR_AUX
#undef XD
  /* Constraint rows and contacts (MJHIP_DATA_EFC / MJHIP_DATA_CONTACT; the reference's
   * d->efc_* arena arrays and d->contact): caller-owned buffers of efc_capacity rows and
   * con_capacity contacts (capacity 0: none kept). A call with skipstage > NONE reads the rows
   * and contacts of the stages it skips from here, as the reference reads the d->efc_* that
   * the preceding mj_forward left (engine_inverse.c:169-192); every call writes back the rows
   * its stages make, with the counts nefc/ne/nf/nl and ncon. */
  int efc_capacity, ne, nf, nl;
  int con_capacity, ncon;
#define XE(type, name, w, stage) type* name;
  MJHIP_DATA_EFC
#undef XE
#define XC(type, name, w, stage) type* name;
  MJHIP_DATA_CONTACT
#undef XC
  /* Compressed Jacobians of sparse-mode models (mj_isSparse: jacobian="sparse", or "auto" with
   * nv >= 60, engine_core_constraint.c:99-106). ten_J (ntendon x nv doubles) and efc_J
   * (efc_capacity x nv doubles) then hold compressed rows as the reference's mjData does
   * (mj_tendon engine_core_smooth.c:651-860; mj_addConstraint engine_core_constraint.c:265-356),
   * described by the arrays below; efc_JT is the transpose (mju_transposeSparse, :2083-2104).
   * Dense-mode models leave them untouched (they may be NULL). */
  int nJ;                   /* nonzeros of efc_J (mjData nJ) */
#define XJ(type, name, dim) type* name;
  MJHIP_DATA_SPARSE
#undef XJ
} mjhipData;

/*---------------------------- status codes of the batch API ------------------------------*/
typedef enum mjhipStatus_ {
  MJHIP_OK              = 0,
  MJHIP_ERR_NO_DEVICE   = -1,   /* no usable HIP device: there is no CPU fallback */
  MJHIP_ERR_ARG         = -2,   /* bad argument (null pointer, size, stage) */
  MJHIP_ERR_HIP         = -3,   /* a HIP runtime call failed; see mjhip_lastError */
  MJHIP_ERR_MODEL       = -4,   /* model uses a feature the device path does not support */
  MJHIP_ERR_CAPACITY    = -5,   /* batch larger than the context capacity */
  MJHIP_ERR_INSTANCE    = 1     /* call completed; at least one instance has a status bit */
} mjhipStatus;

/* flags for mjhipBatchDesc.flags */
#define MJHIP_FLAG_DEVICE_PTRS   (1 << 0)  /* qpos/qvel/qacc/qfrc pointers are device memory */
#define MJHIP_FLAG_MIRROR_INPUT  (1 << 1)  /* inputs already in the device mirror (skip upload) */
#define MJHIP_FLAG_NO_MIRROR     (1 << 2)  /* reserved: write only qfrc_inverse */
#define MJHIP_FLAG_GENERIC       (1 << 3)  /* force the generic (model-data-driven) kernel
                                              even when a straight-line kernel matches */

/* Mirror layout on the device (the "batched SoA mirror" of SURVEY.md §7 L1):
 * every per-instance field F of size S = d0*d1 is stored as
 *     F[(blk*S + k)*64 + lane],  instance = blk*64 + lane,  k = 0..S-1
 * i.e. 64-instance blocks (one wavefront), component-major inside a block, so one
 * wavefront's access to component k of F is one contiguous 512-byte segment.
 * The constraint-row, contact and Jacobian fields (efc_* rows and compressed-row arrays,
 * jar, con_*), which lanes index by their own row or contact counts, are instance-major
 * inside the same 64-instance blocks instead:
 *     F[(blk*64 + lane)*S + k]
 * mjhip_mirrorDownload / mjhip_mirrorUpload hide the difference (one row per instance). */
#define MJHIP_BLOCK 64

/*---------------------------- library / device ---------------------------------------------*/
MJHIP_API const char* mjhip_version(void);
MJHIP_API int mjhip_deviceCount(void);
MJHIP_API const char* mjhip_lastError(void);
/* error callback for the single-instance entry points (mju_user_error analogue);
 * default prints and returns (it never exits the process). */
MJHIP_API void mjhip_setErrorCallback(void (*cb)(const char* msg));

/* size of a per-instance field in doubles (mjxmacro dims), -1 if unknown */
MJHIP_API int mjhip_fieldSize(const mjhipModel* m, const char* name);
/* number of fp64 mjData values written per instance by mj_inverseSkip(skipstage=NONE):
 * W in SURVEY.md §8d (2,563 for the humanoid) */
MJHIP_API int mjhip_outputDoubles(const mjhipModel* m);

/*---------------------------- batched engine -----------------------------------------------*/
typedef struct mjhipContext_ mjhipContext;

/* upload the model to `device` and allocate a mirror for `capacity` instances */
MJHIP_API int mjhip_contextCreate(const mjhipModel* m, int device, int capacity,
                                  mjhipContext** out);
/* mjhip_contextCreate with per-instance caps on contacts and constraint rows (0 = the exact
 * worst case of mjhip_modelCapacity), the analogue of the reference's <size nconmax njmax>
 * / memory arena bound (user_model.cc, mj_makeData): a model whose worst case is far beyond
 * what its states produce (model/humanoid/humanoid100.xml: 16,123 contacts, 68,644 rows of
 * 627 columns) sizes the mirror for what it needs. An instance that exceeds a cap is flagged
 * MJHIP_INST_CNSTRFULL (mjWARN_CONTACTFULL / mjWARN_CNSTRFULL). */
MJHIP_API int mjhip_contextCreateCapped(const mjhipModel* m, int device, int capacity,
                                        int max_contacts, int max_rows, mjhipContext** out);
MJHIP_API void mjhip_contextFree(mjhipContext* c);
MJHIP_API int mjhip_contextCapacity(const mjhipContext* c);
/* name of the straight-line (model-specialized) kernel selected for the context's model by
 * signature, or NULL when the generic kernel runs */
MJHIP_API const char* mjhip_contextFastKernel(const mjhipContext* c);
/* Run-time specialization: load a straight-line kernel generated for this
 * context's model after the library was built. `image` is a gfx950 code object (hipcc
 * --genco of codegen.py's source for the model, mujoco_inversedynamicstest_amd/
 * specialize.py) holding extern "C" k_all_<name>; `signature` is the model signature it was
 * generated for (MJHIP_ERR_MODEL if it is not this model's) and `cmode` its constraint mode
 * (0 none, 1 work-list, 2 every instance). The kernel then serves skipstage = NONE calls
 * exactly as a bundled one does; mjhip_contextFastKernel returns `name`. */
MJHIP_API int mjhip_contextLoadKernel(mjhipContext* c, const void* image, size_t size,
                                      const char* name, unsigned long long signature,
                                      int cmode);
/* kernels the context's last batched mj_inverseSkip ran on: 0 the generic kernel, 1 the
 * straight-line pipeline (skipstage NONE), 2 the straight-line mj_inverseSkip(POS / VEL)
 * kernels (k_va / k_acc of the model's generated code), 3 the straight-line pipeline of a
 * contact model split over two streams (position stage, then the cooperative constraint
 * kernel beside the fac / va stages, joined by the assembly; opt-in with MJHIP_SPLIT=1);
 * -1 before any call */
MJHIP_API int mjhip_contextLastPath(const mjhipContext* c);
/* the constraint kernel the context's last straight-line call launched, e.g.
 * "k_constraint_coop<16, false, true, false>" (the work-list kernel of a limits-only model) or
 * "k_constraint<true, true, false>"; "none" when it launched none (profiles name it) */
MJHIP_API const char* mjhip_contextConstraintKernel(const mjhipContext* c);
/* instances of the last fast-path call that had active constraint rows and were recomputed
 * by the generic kernel (blocking read; -1 on error) */
MJHIP_API int mjhip_worklistCount(mjhipContext* c);
/* HIP stream used by the context (hipStream_t as void*); may be replaced by the caller */
MJHIP_API void* mjhip_contextStream(mjhipContext* c);
MJHIP_API int mjhip_contextSetStream(mjhipContext* c, void* stream);

/* Batched mj_inverseSkip over B instances of one model.
 * qpos (B x nq), qvel (B x nv), qacc (B x nv) in, qfrc_inverse (B x nv) out: row-major,
 * one row per instance (the layout of rollout.cc's state arrays). Host pointers unless
 * MJHIP_FLAG_DEVICE_PTRS. qfrc_inverse may be NULL (result stays in the mirror).
 * skipstage/skipsensor have the reference semantics (engine_inverse.c:197-261); with
 * skipstage > NONE the earlier-stage fields must already be in the mirror (a previous
 * call on the same context, or mjhip_mirrorUpload). status (B ints, host) may be NULL.
 * Asynchronous w.r.t. the host only with MJHIP_FLAG_DEVICE_PTRS. */
MJHIP_API int mjhip_inverseBatch(mjhipContext* c, int B,
                                 const mjtNum* qpos, const mjtNum* qvel, const mjtNum* qacc,
                                 mjtNum* qfrc_inverse, int skipstage, int skipsensor,
                                 int flags, int* status);

/* Batched mj_forward (engine_forward.c:1054-1090 order: fwdPosition, fwdVelocity,
 * fwdActuation, fwdAcceleration, fwdConstraint) for constraint-free states: qacc =
 * qacc_smooth = M^-1 (qfrc_passive - qfrc_bias + qfrc_applied + qfrc_actuator + J'xfrc).
 * The constraint solver is not implemented: an instance with constraint rows is flagged
 * MJHIP_INST_UNSUPPORTED (its qacc is qacc_smooth). qpos/qvel (B x nq, B x nv) and optional
 * ctrl (B x nu) are row-major inputs unless MJHIP_FLAG_MIRROR_INPUT; qfrc_applied and
 * xfrc_applied are read from the mirror (mjhip_mirrorUpload; zero after context creation).
 * Optional qacc (B x nv) receives the result; every mjData field is in the mirror. */
MJHIP_API int mjhip_forwardBatch(mjhipContext* c, int B, const mjtNum* qpos, const mjtNum* qvel,
                                 const mjtNum* ctrl, mjtNum* qacc, int flags, int* status);

/* copy one mirror field (reference name) of instances [first, first+count) to/from host
 * memory in the reference's per-instance row-major layout (count x fieldSize) */
MJHIP_API int mjhip_mirrorDownload(mjhipContext* c, const char* field, int first, int count,
                                   mjtNum* dst);

/* Int per-instance arrays of the device path: the reference's mjData int arrays on this path
 * (efc_type, efc_id, efc_state; contact dim/geom/exclude/efc_address as con_*) and the counts
 * efc_count = {nefc, ne, nf, nl}, con_count = {ncon}. Rows of mjhip_fieldSizeInt() ints. */
MJHIP_API int mjhip_mirrorDownloadInt(mjhipContext* c, const char* field, int first, int count,
                                      int* dst);
MJHIP_API int mjhip_fieldSizeInt(const mjhipContext* c, const char* field);
/* doubles per instance of any fp64 mirror field of this context: the mjData fields and the
 * device path's per-instance arrays (efc_* rows, con_* contacts); -1 if unknown */
MJHIP_API int mjhip_mirrorFieldSize(const mjhipContext* c, const char* field);
MJHIP_API int mjhip_mirrorUpload(mjhipContext* c, const char* field, int first, int count,
                                 const mjtNum* src);
/* device pointer of a mirror field (block layout above) */
MJHIP_API void* mjhip_mirrorDevicePtr(mjhipContext* c, const char* field);
/* per-instance status words of the last call (device pointer, B ints) */
MJHIP_API int mjhip_statusDownload(mjhipContext* c, int first, int count, int* dst);

/* Batched mjd_inverseFD (engine_derivative_fd.c:611-719, mujoco.h:1244-1247) with
 * flg_actuation = 0: for each of B base states, forward differences with step eps of
 * qfrc_inverse w.r.t. qacc (DfDa), qvel (DfDv) and qpos (DfDq, via mj_integratePos), each
 * nv x nv in the reference's transposed layout; of sensordata (DsDq/DsDv/DsDa, nv x
 * nsensordata, sensors skipped when all three are NULL); of qM (DmDq, nv x nM). Every
 * output may be NULL. Per base state the outputs are consecutive (B x nv x n row-major);
 * host pointers unless MJHIP_FLAG_DEVICE_PTRS. Same argument order as the reference. */
MJHIP_API int mjhip_inverseFDBatch(mjhipContext* c, int B,
                                   const mjtNum* qpos, const mjtNum* qvel, const mjtNum* qacc,
                                   mjtNum eps, mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa,
                                   mjtNum* DsDq, mjtNum* DsDv, mjtNum* DsDa, mjtNum* DmDq,
                                   int flags);

/* mjhip_inverseFDBatch with the reference's flg_actuation (engine_derivative_fd.c:160-168):
 * when set, every evaluation's force is qfrc_inverse - qfrc_actuator (mj_fwdActuation of the
 * base state's controls `ctrl`, B x nu, which may be NULL when nu == 0). Actuators with
 * activation dynamics or muscle/user gain and bias are MJHIP_ERR_MODEL. */
MJHIP_API int mjhip_inverseFDBatchEx(mjhipContext* c, int B, const mjtNum* qpos,
                                     const mjtNum* qvel, const mjtNum* qacc, const mjtNum* ctrl,
                                     mjtNum eps, int flg_actuation, mjtNum* DfDq, mjtNum* DfDv,
                                     mjtNum* DfDa, mjtNum* DsDq, mjtNum* DsDv, mjtNum* DsDa,
                                     mjtNum* DmDq, int flags);

/* Per-instance row capacities of a model on the device path: constraint rows (efc) and
 * contacts an instance can produce (exact upper bounds for the implemented functions). Size
 * mjhipData's efc_* / con_* buffers with these. */
MJHIP_API int mjhip_modelCapacity(const mjhipModel* m, int* efc_rows, int* contacts);

/* mjc_ccd (engine_collision_gjk.c:2215-2343; MJAPI, engine_collision_gjk.h:92), the native
 * GJK/EPA solver, over n geom pairs of the context's model, one device lane per pair. Pair i
 * is geoms g1[i], g2[i] at the caller's frames pos1/pos2 (n x 3) and mat1/mat2 (n x 9,
 * row-major geom_xmat), both inflated by margin[i] (mjc_initCCDObj's margin; NULL: 0), with
 * the mjCCDConfig {max_iterations, tolerance, max_contacts, dist_cutoff}. max_contacts 0 asks
 * for the distance alone (no penetration recovery), 1 for one contact, more for the
 * multicontact polygon of a penetrating box / mesh pair (gjk.c:1460-2193; mesh polygons from
 * the compiler, mjCMesh::MakePolygons). Outputs (host arrays):
 * dist[n] (mjc_ccd's return value), nx[n] (status.nx), x1/x2 (n x xcap x 3, status.x1/x2: the
 * witness points, xcap = max(1, min(max_contacts, mjMAXCONPAIR = 50))). Status codes as
 * everywhere; MJHIP_ERR_MODEL when a pair's polytope outgrew the solver's face capacity or
 * needs multicontact beyond the device's polygon capacity (a mesh polygon of more than 16
 * vertices, or a vertex on more than 16 polygons; the reference allows 150). */
MJHIP_API int mjhip_ccdBatch(mjhipContext* c, int n, const int* g1, const int* g2,
                             const mjtNum* pos1, const mjtNum* mat1, const mjtNum* pos2,
                             const mjtNum* mat2, const mjtNum* margin, int max_iterations,
                             mjtNum tolerance, int max_contacts, mjtNum dist_cutoff,
                             mjtNum* dist, int* nx, mjtNum* x1, mjtNum* x2);

/* Time `reps` back-to-back launches of the fused inverse kernel on the context's stream
 * with HIP events (device-resident mirror inputs, B instances). Writes the average
 * milliseconds per launch to *ms. Used by bench.py for the roofline figure. */
MJHIP_API int mjhip_timeInverseKernel(mjhipContext* c, int B, int reps, int skipstage,
                                      int flags, float* ms);

/* Per-stage timers: the reference's mjtTimer slots (include/mujoco/mjdata.h) and mjTimerStat,
 * which mj_invPosition, mj_invConstraint and mj_inverseSkip accumulate
 * (engine_inverse.c:38-67, :170-191, :199-260). With timers on (mjhip_contextTimers),
 * every mjhip_inverseBatch call of the context adds to them:
 *   INVERSE         device wall time of the call (HIP events on its stream, milliseconds)
 *   POSITION        POS_KINEMATICS + POS_INERTIA + POS_COLLISION + POS_MAKE
 *   POS_KINEMATICS  kinematics, comPos, camlight, tendons, transmission (the straight-line
 *                   kernels' position stage, which also forms qM by crb)
 *   POS_INERTIA     crb + factorM (factorM alone on the straight-line path)
 *   POS_COLLISION   mj_collision          POS_MAKE    mj_makeConstraint
 *   VELOCITY        mj_invVelocity (comVel, passive, RNE bias; the straight-line kernels'
 *                   velocity stage, RNE with qacc included)
 *   CONSTRAINT      mj_discreteAcc + mj_invConstraint (reference, update, J'force)
 * Stage durations are the mean wall time (the 100 MHz device clock) a wavefront of 64
 * instances spends in the stage, in milliseconds; `number` counts the calls. The phase marks
 * are read by lane 0 of each wave: timed calls synchronize the stream, and one context per
 * process is timed at a time. */
typedef enum mjhipTimer_ {
  mjhipTIMER_STEP = 0, mjhipTIMER_FORWARD, mjhipTIMER_INVERSE, mjhipTIMER_POSITION,
  mjhipTIMER_VELOCITY, mjhipTIMER_ACTUATION, mjhipTIMER_CONSTRAINT, mjhipTIMER_ADVANCE,
  mjhipTIMER_POS_KINEMATICS, mjhipTIMER_POS_INERTIA, mjhipTIMER_POS_COLLISION,
  mjhipTIMER_POS_MAKE, mjhipTIMER_POS_PROJECT, mjhipTIMER_COL_BROAD, mjhipTIMER_COL_NARROW,
  mjhipNTIMER
} mjhipTimer;
typedef struct mjhipTimerStat_ {
  mjtNum duration;                  /* accumulated milliseconds */
  int number;                       /* number of calls */
} mjhipTimerStat;
/* enable != 0: allocate the accumulator and time the following calls; 0: stop timing */
MJHIP_API int mjhip_contextTimers(mjhipContext* c, int enable);
/* copy the mjhipNTIMER slots to out; reset != 0 clears them afterwards */
MJHIP_API int mjhip_timerRead(mjhipContext* c, mjhipTimerStat* out, int reset);

/*---------------------------- single-instance drop-in -------------------------------------*/
/* Same semantics and outputs as the reference functions of the same name (engine_inverse.c,
 * engine_core_smooth.c, engine_support.c, engine_derivative_fd.c); they run one instance on
 * the GPU (device 0 unless mjhip_setDevice). Each uploads the fields of d the reference
 * function reads -- for mj_inverseSkip(skipstage) the inputs, the outputs of the skipped
 * stages and their constraint rows / contacts (d->nefc, ne, nf, nl, ncon and the efc_* /
 * con_* arrays) -- and writes back exactly the fields the reference function writes,
 * including the rows of the stages that ran. Device state is cached per model content
 * (at most 16 models, least recently used released first). Errors go to the error
 * callback (or stderr); per-instance conditions to d->status. */
MJHIP_API void mjhip_setDevice(int device);
MJHIP_API void mjhip_inverse(const mjhipModel* m, mjhipData* d);
MJHIP_API void mjhip_inverseSkip(const mjhipModel* m, mjhipData* d, int skipstage,
                                 int skipsensor);
MJHIP_API void mjhip_invPosition(const mjhipModel* m, mjhipData* d);
MJHIP_API void mjhip_invVelocity(const mjhipModel* m, mjhipData* d);
MJHIP_API void mjhip_invConstraint(const mjhipModel* m, mjhipData* d);
MJHIP_API void mjhip_rne(const mjhipModel* m, mjhipData* d, int flg_acc, mjtNum* result);
/* mj_xfrcAccumulate (engine_support.c:1254-1261): qfrc += J' xfrc_applied over bodies 1..
 * nbody-1, from d's xipos, subtree_com and cdof */
MJHIP_API void mjhip_xfrcAccumulate(const mjhipModel* m, mjhipData* d, mjtNum* qfrc);
/* mj_compareFwdInv (engine_inverse.c:275-316): from a forward pass's state and constraint
 * rows in d, solver_fwdinv = (|qfrc_constraint fwd - inv|, |qfrc_applied + qfrc_actuator +
 * J'xfrc_applied - qfrc_inverse|); qfrc_constraint and efc_force keep the forward values */
MJHIP_API void mjhip_compareFwdInv(const mjhipModel* m, mjhipData* d);
/* mjd_inverseFD (engine_derivative_fd.c:611-719) for one mjData; d keeps its qpos/qvel/qacc
 * and holds the outputs of the reference's last evaluation afterwards */
MJHIP_API void mjhip_inverseFD(const mjhipModel* m, mjhipData* d, mjtNum eps,
                               mjtByte flg_actuation, mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa,
                               mjtNum* DsDq, mjtNum* DsDv, mjtNum* DsDa, mjtNum* DmDq);
/* release the per-model device state cached by the single-instance entry points */
MJHIP_API void mjhip_releaseModel(const mjhipModel* m);

#ifdef __cplusplus
}
#endif

#endif  /* MJHIP_H_ */
