/* engine_inverse_mjhip.c — reference-side adapter: replaces src/engine/engine_inverse.c of
 * fancifulland2718/mujoco_InverseDynamicsTest (MuJoCo 3.3.1) so that mj_inverse,
 * mj_inverseSkip, mj_invPosition, mj_invVelocity, mj_invConstraint and mj_compareFwdInv run
 * on the MI355X through libmjhip.so (include/mjhip.h).
 *
 * mjhipModel/mjhipData use the reference's field names, element types and row-major
 * shapes, so the views below are plain pointer copies generated from the same X-macro
 * tables (include/mjhip_fields.h); a name or type mismatch with mjModel/mjData is a
 * compile error (tests/test_integration.py compiles this file against the reference's
 * public headers, tests/test_adapter_exec.py runs it on real mjModel/mjData structs).
 *
 * Constraint rows and contacts. The reference keeps them in the mjData arena: mj_collision
 * resets it and lays the contacts at its start (engine_collision_driver.c:265-285), and
 * mj_makeConstraint allocates the efc arrays behind them (engine_core_constraint.c:50-80,
 * :2003-2075). Calls that skip the position stage read those rows in place (the efc arrays
 * are structure-of-arrays like mjhipData's; contacts are converted from mjContact). Calls
 * that run the position stage get the rows back in capacity-sized staging buffers and the
 * adapter re-creates the arena layout the reference would have left: contacts at the arena
 * start, then every MJDATA_ARENA_POINTERS_SOLVER array of the counted size, tendon_efcadr
 * included (rules of engine_core_constraint.c:668-671, :811-814, :949-952).
 *
 * Sparse-Jacobian models (mj_isSparse, engine_core_constraint.c:99-106: jacobian="sparse",
 * or "auto" with nv >= 60) get the reference's compressed layout: ten_J and its
 * rownnz/rowadr/colind in place in mjData, and in the arena efc_J/efc_JT over nJ entries with
 * their rownnz/rowadr/colind, and the row supernodes mj_makeConstraint derives from them
 * (:2083-2104, mju_superSparse engine_util_sparse.c:520-550, restated below).
 *
 * Models are checked for features the device path does not implement and which mjhipModel
 * does not carry (flexes, plugins, muscle/user actuator gains and biases, an affine velocity
 * gain with activation dynamics, SDF geoms; adapter_unsupported): such a model is an
 * mju_error, never a silently different result. Predefined <contact><pair>s are carried.
 *
 * Build (in the reference tree): drop engine_inverse.c from src/engine/CMakeLists.txt,
 * add this file, add <repo>/include to the include path and link libmjhip.so.
 */
#include <stdlib.h>
#include <string.h>

#include <mujoco/mujoco.h>
#include <mujoco/mjxmacro.h>

#include "mjhip.h"

/* engine_io.h (MJAPI, not in the public headers) */
void* mj_arenaAllocByte(mjData* d, size_t bytes, size_t alignment);

/*------------------------------------------------------------------ model --------------*/

/* features outside the device subset that mjhipModel cannot show; NULL when supported */
static const char* adapter_unsupported(const mjModel* m) {
  if (m->nflex) return "flexes";
  if (m->nplugin) return "plugins";
  for (int i = 0; i < m->nu; i++) {
    /* mjd_actuator_vel reads mjData.act for these (engine_derivative.c:855-863) */
    if (m->actuator_dyntype[i] != mjDYN_NONE && m->actuator_gaintype[i] == mjGAIN_AFFINE &&
        m->actuator_gainprm[mjNGAIN*i + 2] != 0) {
      return "an affine velocity gain with activation dynamics";
    }
    if (m->actuator_gaintype[i] >= mjGAIN_MUSCLE || m->actuator_biastype[i] >= mjBIAS_MUSCLE) {
      return "muscle or user actuator gain/bias";
    }
  }
  for (int i = 0; i < m->ngeom; i++) {
    if (m->geom_type[i] == mjGEOM_SDF) return "SDF geoms";
  }
  return NULL;
}

/* the mjhipModel view of m, rebuilt per call: the library keys its device state on the
 * model's content, so nothing here caches by address */
static void model_view(const mjModel* m, const mjData* d, mjhipModel* hm) {
  const char* why = adapter_unsupported(m);
  if (why) mju_error("mjhip: model uses %s, which the MI355X inverse path does not implement",
                     why);
  memset(hm, 0, sizeof(*hm));
#define XS(name) hm->name = m->name;
  MJHIP_MODEL_SIZES
#undef XS
  hm->opt.timestep = m->opt.timestep;
  hm->opt.impratio = m->opt.impratio;
  memcpy(hm->opt.gravity, m->opt.gravity, sizeof(hm->opt.gravity));
  memcpy(hm->opt.wind, m->opt.wind, sizeof(hm->opt.wind));
  memcpy(hm->opt.magnetic, m->opt.magnetic, sizeof(hm->opt.magnetic));
  hm->opt.density = m->opt.density;
  hm->opt.viscosity = m->opt.viscosity;
  hm->opt.o_margin = m->opt.o_margin;
  memcpy(hm->opt.o_solref, m->opt.o_solref, sizeof(hm->opt.o_solref));
  memcpy(hm->opt.o_solimp, m->opt.o_solimp, sizeof(hm->opt.o_solimp));
  memcpy(hm->opt.o_friction, m->opt.o_friction, sizeof(hm->opt.o_friction));
  hm->opt.ccd_tolerance = m->opt.ccd_tolerance;
  hm->opt.ccd_iterations = m->opt.ccd_iterations;
  hm->opt.integrator = m->opt.integrator;
  hm->opt.cone = m->opt.cone;
  hm->opt.jacobian = m->opt.jacobian;
  hm->opt.disableflags = m->opt.disableflags;
  hm->opt.enableflags = m->opt.enableflags;
  /* arrays that live in mjModel */
#define X(type, name, d0, d1) hm->name = m->name;
  MJHIP_MODEL_POINTERS_M
#undef X
  /* model-constant sparse structures that live in mjData in the reference */
#define X(type, name, d0, d1) hm->name = d->name;
  MJHIP_MODEL_POINTERS_D
#undef X
}

/*------------------------------------------------------------------ data ---------------*/

/* mj_isSparse (engine_core_constraint.c:99-106) */
static int is_sparse(const mjModel* m) {
  return m->opt.jacobian == mjJAC_SPARSE || (m->opt.jacobian == mjJAC_AUTO && m->nv >= 60);
}

/* mju_superSparse (engine_util_sparse.c:520-550): rowsuper[r] = how many following rows share
 * row r's pattern */
static void super_sparse(int nr, int* rowsuper, const int* rownnz, const int* rowadr,
                         const int* colind) {
  if (!nr) return;
  for (int r = 0; r < nr-1; r++) {
    rowsuper[r] = rownnz[r] == rownnz[r+1] &&
                  !memcmp(colind + rowadr[r], colind + rowadr[r+1], rownnz[r]*sizeof(int));
  }
  rowsuper[nr-1] = 0;
  for (int r = nr-2; r >= 0; r--) {
    if (rowsuper[r]) rowsuper[r] += rowsuper[r+1];
  }
}

/* per-call view of d plus the staging it needs */
typedef struct {
  mjhipData hd;
  void* stage;          /* malloc'd row/contact staging (one block), or NULL */
} DataView;

static void data_fields(mjData* d, mjhipData* hd) {
  memset(hd, 0, sizeof(*hd));
  memcpy(hd->energy, d->energy, sizeof(hd->energy));
  hd->time = d->time;
#define XD(name, d0, d1, stage) hd->name = d->name;
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
  MJHIP_DATA_SENSOR_AUX
#undef XD
  /* the tendon Jacobian's compressed structure (used by sparse-mode models) */
  hd->ten_J_rownnz = d->ten_J_rownnz;
  hd->ten_J_rowadr = d->ten_J_rowadr;
  hd->ten_J_colind = d->ten_J_colind;
}

/* bytes per row of the efc arrays of MJHIP_DATA_SPARSE (rows x 1 or rows x nv) plus the two
 * nv-sized ones, for a sparse-mode model's staging */
static size_t sparse_bytes(const mjModel* m, int rows) {
  return sizeof(int) * (size_t)rows * (2 + 2*(size_t)m->nv) + sizeof(mjtNum) * (size_t)rows *
         m->nv + sizeof(int) * 2 * (size_t)m->nv + 8*8;
}

/* bytes of one row (XE) / one contact (XC) over every array */
static size_t row_bytes(const mjModel* m) {
  size_t b = 0;
#undef MJ_M
#define MJ_M(n) m->n
#define XE(type, name, w, stage) b += sizeof(type) * (size_t)(w);
  MJHIP_DATA_EFC
#undef XE
#undef MJ_M
#define MJ_M(n) n
  return b;
}

static size_t contact_bytes(void) {
  size_t b = 0;
#define XC(type, name, w, stage) b += sizeof(type) * (size_t)(w);
  MJHIP_DATA_CONTACT
#undef XC
  return b;
}

/* contacts: mjContact (AoS) <-> mjhipData con_* (SoA) */
static void contacts_to_soa(const mjData* d, mjhipData* hd) {
  for (int i = 0; i < d->ncon; i++) {
    const mjContact* c = d->contact + i;
    hd->con_dist[i] = c->dist;
    memcpy(hd->con_pos + 3*i, c->pos, 3*sizeof(mjtNum));
    memcpy(hd->con_frame + 9*i, c->frame, 9*sizeof(mjtNum));
    hd->con_includemargin[i] = c->includemargin;
    memcpy(hd->con_friction + 5*i, c->friction, 5*sizeof(mjtNum));
    memcpy(hd->con_solref + 2*i, c->solref, 2*sizeof(mjtNum));
    memcpy(hd->con_solreffriction + 2*i, c->solreffriction, 2*sizeof(mjtNum));
    memcpy(hd->con_solimp + 5*i, c->solimp, 5*sizeof(mjtNum));
    hd->con_mu[i] = c->mu;
    hd->con_dim[i] = c->dim;
    hd->con_geom[2*i] = c->geom[0];
    hd->con_geom[2*i+1] = c->geom[1];
    hd->con_exclude[i] = c->exclude;
    hd->con_efc_address[i] = c->efc_address;
  }
}

static void contact_from_soa(const mjhipData* hd, int i, mjContact* c) {
  memset(c, 0, sizeof(*c));
  c->dist = hd->con_dist[i];
  memcpy(c->pos, hd->con_pos + 3*i, 3*sizeof(mjtNum));
  memcpy(c->frame, hd->con_frame + 9*i, 9*sizeof(mjtNum));
  c->includemargin = hd->con_includemargin[i];
  memcpy(c->friction, hd->con_friction + 5*i, 5*sizeof(mjtNum));
  memcpy(c->solref, hd->con_solref + 2*i, 2*sizeof(mjtNum));
  memcpy(c->solreffriction, hd->con_solreffriction + 2*i, 2*sizeof(mjtNum));
  memcpy(c->solimp, hd->con_solimp + 5*i, 5*sizeof(mjtNum));
  c->mu = hd->con_mu[i];
  c->dim = hd->con_dim[i];
  c->geom[0] = c->geom1 = hd->con_geom[2*i];
  c->geom[1] = c->geom2 = hd->con_geom[2*i+1];
  c->flex[0] = c->flex[1] = -1;
  c->elem[0] = c->elem[1] = -1;
  c->vert[0] = c->vert[1] = -1;
  c->exclude = hd->con_exclude[i];
  c->efc_address = hd->con_efc_address[i];
}

/* carve the XE arrays of `rows` rows and/or the XC arrays of `cons` contacts out of one
 * block, each array 8-byte aligned */
static void* stage_alloc(const mjModel* m, mjhipData* hd, int rows, int cons, int efc,
                         int con) {
  size_t total = (efc ? row_bytes(m) * (size_t)rows : 0) +
                 (con ? contact_bytes() * (size_t)cons : 0) + 8*64 +
                 (efc && is_sparse(m) ? sparse_bytes(m, rows) : 0);
  char* p = (char*)malloc(total);
  if (!p) mju_error("mjhip: out of host memory for %d constraint rows", rows);
  char* q = p;
#undef MJ_M
#define MJ_M(n) m->n
  if (efc) {
    hd->efc_capacity = rows;
#define XE(type, name, w, stage) \
    hd->name = (type*)q; q += (sizeof(type) * (size_t)(w) * rows + 7) & ~(size_t)7;
    MJHIP_DATA_EFC
#undef XE
    if (is_sparse(m)) {
      const size_t rn = (size_t)rows * m->nv;
#define CARVE(name, type, n) hd->name = (type*)q; q += (sizeof(type) * (n) + 7) & ~(size_t)7;
      CARVE(efc_J_rownnz, int, (size_t)rows)
      CARVE(efc_J_rowadr, int, (size_t)rows)
      CARVE(efc_J_colind, int, rn)
      CARVE(efc_JT, mjtNum, rn)
      CARVE(efc_JT_rownnz, int, (size_t)m->nv)
      CARVE(efc_JT_rowadr, int, (size_t)m->nv)
      CARVE(efc_JT_colind, int, rn)
#undef CARVE
    }
  }
  if (con) {
    hd->con_capacity = cons;
#define XC(type, name, w, stage) \
    hd->name = (type*)q; q += (sizeof(type) * (size_t)(w) * cons + 7) & ~(size_t)7;
    MJHIP_DATA_CONTACT
#undef XC
  }
#undef MJ_M
#define MJ_M(n) n
  return p;
}

/* the view for a call that reads the rows of d (skips the position stage): efc arrays in
 * place, contacts converted into staging */
static void view_existing_rows(const mjModel* m, mjData* d, DataView* v) {
  data_fields(d, &v->hd);
  mjhipData* hd = &v->hd;
  hd->nefc = d->nefc;
  hd->ne = d->ne;
  hd->nf = d->nf;
  hd->nl = d->nl;
  hd->ncon = d->ncon;
  hd->efc_capacity = d->nefc;
#define XE(type, name, w, stage) hd->name = d->name;
  MJHIP_DATA_EFC
#undef XE
  /* compressed rows of a sparse-mode model, in place in the arena */
  hd->nJ = d->nJ;
  hd->efc_J_rownnz = d->efc_J_rownnz;
  hd->efc_J_rowadr = d->efc_J_rowadr;
  hd->efc_J_colind = d->efc_J_colind;
  hd->efc_JT = d->efc_JT;
  hd->efc_JT_rownnz = d->efc_JT_rownnz;
  hd->efc_JT_rowadr = d->efc_JT_rowadr;
  hd->efc_JT_colind = d->efc_JT_colind;
  v->stage = d->ncon ? stage_alloc(m, hd, 0, d->ncon, 0, 1) : NULL;
  if (d->ncon) contacts_to_soa(d, hd);
}

/* the view for a call that makes the rows (runs the position stage): capacity staging */
static void view_new_rows(const mjModel* m, const mjhipModel* hm, mjData* d, DataView* v) {
  data_fields(d, &v->hd);
  int rows = 0, cons = 0;
  mjhip_modelCapacity(hm, &rows, &cons);
  v->stage = stage_alloc(m, &v->hd, rows, cons, 1, 1);
}

/* mj_clearEfc (engine_io.h:156-163): every arena array invalidated, contacts kept at the
 * arena start */
static void clear_efc(mjData* d) {
#define X(type, name, nr, nc) d->name = NULL;
  MJDATA_ARENA_POINTERS
#undef X
  d->nefc = 0;
  d->nisland = 0;
  d->contact = (mjContact*)d->arena;
}

/* d's arena as mj_collision + mj_makeConstraint leave it, filled from the staged rows */
static void arena_from_rows(const mjModel* m, mjData* d, const mjhipData* hd) {
  /* mj_collision: reset the arena and the efc arrays (engine_collision_driver.c:270-273) */
  d->ncon = 0;
  d->parena = 0;
  clear_efc(d);
  d->ne = d->nf = d->nl = d->nJ = d->nA = 0;
  /* mj_addContact (engine_core_constraint.c:234-260), one contact at a time at the arena
   * start; one that does not fit (nconmax or the arena) is dropped with mjWARN_CONTACTFULL */
  int dropped = 0;
  for (int i = 0; i < hd->ncon; i++) {
    mjContact* c = NULL;
    if (m->nconmax == -1 || d->ncon < m->nconmax) {
      d->parena = d->ncon * sizeof(mjContact);
      c = (mjContact*)mj_arenaAllocByte(d, sizeof(mjContact), _Alignof(mjContact));
    }
    if (!c) {
      mj_warning(d, mjWARN_CONTACTFULL, d->ncon);
      dropped++;
      continue;
    }
    contact_from_soa(hd, i, c);
    d->ncon++;
  }
  /* mj_makeConstraint (engine_core_constraint.c:2005-2075): sizes, then arenaAllocEfc
   * (:50-80) with the dense Jacobian */
  if (m->opt.disableflags & mjDSBL_CONSTRAINT) return;
  const int nefc = hd->nefc, sparse = is_sparse(m);
  d->nJ = sparse ? hd->nJ : nefc * m->nv;
  d->nefc = nefc;
  d->parena = d->ncon * sizeof(mjContact);
  /* the device made rows for every contact: with contacts dropped they are not the rows the
   * reference would make, so the efc arrays are treated as not fitting either */
  int ok = !dropped;
#undef MJ_M
#define MJ_M(n) m->n
#undef MJ_D
#define MJ_D(n) d->n
#define X(type, name, nr, nc)                                                   \
  if (ok) {                                                                     \
    d->name = mj_arenaAllocByte(d, sizeof(type) * (nr) * (nc), _Alignof(type)); \
    if (!d->name) ok = 0;                                                       \
  }
  MJDATA_ARENA_POINTERS_SOLVER
#undef X
#undef MJ_D
#define MJ_D(n) n
  if (!ok) {
    mj_warning(d, mjWARN_CNSTRFULL, (int)d->narena);
    clear_efc(d);
    d->parena = d->ncon * sizeof(mjContact);
    return;
  }
  d->ne = hd->ne;
  d->nf = hd->nf;
  d->nl = hd->nl;
#define XE(type, name, w, stage) \
  memcpy(d->name, hd->name, sparse && !strcmp(#name, "efc_J") ? sizeof(type) * (size_t)d->nJ \
                                                                : sizeof(type) * (size_t)(w) * nefc);
  MJHIP_DATA_EFC
#undef XE
#undef MJ_M
#define MJ_M(n) n
  if (sparse && nefc) {
    /* :2083-2104: the transpose, the rows' and the transpose's supernodes */
    memcpy(d->efc_J_rownnz, hd->efc_J_rownnz, sizeof(int) * nefc);
    memcpy(d->efc_J_rowadr, hd->efc_J_rowadr, sizeof(int) * nefc);
    memcpy(d->efc_J_colind, hd->efc_J_colind, sizeof(int) * d->nJ);
    memcpy(d->efc_JT, hd->efc_JT, sizeof(mjtNum) * d->nJ);
    memcpy(d->efc_JT_rownnz, hd->efc_JT_rownnz, sizeof(int) * m->nv);
    memcpy(d->efc_JT_rowadr, hd->efc_JT_rowadr, sizeof(int) * m->nv);
    memcpy(d->efc_JT_colind, hd->efc_JT_colind, sizeof(int) * d->nJ);
    super_sparse(nefc, d->efc_J_rowsuper, d->efc_J_rownnz, d->efc_J_rowadr, d->efc_J_colind);
    super_sparse(m->nv, d->efc_JT_rowsuper, d->efc_JT_rownnz, d->efc_JT_rowadr,
                 d->efc_JT_colind);
  }
  d->maxuse_con = d->maxuse_con > d->ncon ? d->maxuse_con : d->ncon;
  d->maxuse_efc = d->maxuse_efc > nefc ? d->maxuse_efc : nefc;
  /* tendon_efcadr: tendon equalities record the equality id, tendon friction and limit rows
   * their first row (engine_core_constraint.c:668-671, :811-814, :949-952) */
  for (int i = 0; i < m->ntendon; i++) d->tendon_efcadr[i] = -1;
  for (int r = 0; r < nefc; r++) {
    const int type = d->efc_type[r], id = d->efc_id[r];
    if (type == mjCNSTR_EQUALITY && m->eq_type[id] == mjEQ_TENDON &&
        (r == 0 || d->efc_type[r-1] != mjCNSTR_EQUALITY || d->efc_id[r-1] != id)) {
      const int t1 = m->eq_obj1id[id], t2 = m->eq_obj2id[id];
      if (d->tendon_efcadr[t1] == -1) d->tendon_efcadr[t1] = id;
      if (t2 >= 0 && d->tendon_efcadr[t2] == -1) d->tendon_efcadr[t2] = id;
    } else if (type == mjCNSTR_FRICTION_TENDON || type == mjCNSTR_LIMIT_TENDON) {
      if (d->tendon_efcadr[id] == -1) d->tendon_efcadr[id] = r;
    }
  }
}

/* outputs held by value in mjhipData, the staging, and the per-instance status. Rows that
 * a stage wrote on rows d already held went straight into d's arrays. */
static void finish(mjData* d, DataView* v) {
  const mjhipData* hd = &v->hd;
  d->solver_fwdinv[0] = hd->solver_fwdinv[0];
  d->solver_fwdinv[1] = hd->solver_fwdinv[1];
  memcpy(d->energy, hd->energy, sizeof(d->energy));
  free(v->stage);
  v->stage = NULL;
  if (hd->status & MJHIP_INST_UNSUPPORTED) {
    mju_error("mjhip: the state needs a collision function the MI355X path does not "
              "implement (status %#x)", (unsigned)hd->status);
  }
  if (hd->status & MJHIP_INST_CNSTRFULL) mj_warning(d, mjWARN_CNSTRFULL, hd->nefc);
}

/*------------------------------------------------------------------ API ----------------*/

void mj_inverseSkip(const mjModel* m, mjData* d, int skipstage, int skipsensor) {
  mjhipModel hm;
  model_view(m, d, &hm);
  DataView v;
  if (skipstage >= mjSTAGE_POS) {
    view_existing_rows(m, d, &v);
  } else {
    view_new_rows(m, &hm, d, &v);
  }
  mjhip_inverseSkip(&hm, &v.hd, skipstage, skipsensor);
  if (skipstage < mjSTAGE_POS) arena_from_rows(m, d, &v.hd);
  finish(d, &v);
}

void mj_inverse(const mjModel* m, mjData* d) {
  mj_inverseSkip(m, d, mjSTAGE_NONE, 0);
}

void mj_invPosition(const mjModel* m, mjData* d) {
  mjhipModel hm;
  model_view(m, d, &hm);
  DataView v;
  view_new_rows(m, &hm, d, &v);
  mjhip_invPosition(&hm, &v.hd);
  arena_from_rows(m, d, &v.hd);
  finish(d, &v);
}

void mj_invVelocity(const mjModel* m, mjData* d) {
  mjhipModel hm;
  model_view(m, d, &hm);
  DataView v;
  view_existing_rows(m, d, &v);
  mjhip_invVelocity(&hm, &v.hd);
  finish(d, &v);
}

void mj_invConstraint(const mjModel* m, mjData* d) {
  mjhipModel hm;
  model_view(m, d, &hm);
  DataView v;
  view_existing_rows(m, d, &v);
  mjhip_invConstraint(&hm, &v.hd);
  finish(d, &v);
}

void mj_compareFwdInv(const mjModel* m, mjData* d) {
  mjhipModel hm;
  model_view(m, d, &hm);
  DataView v;
  view_existing_rows(m, d, &v);
  mjhip_compareFwdInv(&hm, &v.hd);
  finish(d, &v);
}

/* The batched derivative path for callers that want it (mjd_inverseFD itself lives in
 * engine_derivative_fd.c and reaches the device through mj_inverseSkip above, one
 * evaluation per call): same arguments as mjd_inverseFD (engine_derivative_fd.c:611-719),
 * all 3nv+1 evaluations in one device batch. */
void mjd_inverseFD_mjhip(const mjModel* m, mjData* d, mjtNum eps, mjtByte flg_actuation,
                         mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa, mjtNum* DsDq, mjtNum* DsDv,
                         mjtNum* DsDa, mjtNum* DmDq) {
  if (m->opt.integrator == mjINT_RK4) mju_error("RK4 integrator is not supported");
  if (m->opt.noslip_iterations) mju_error("noslip solver is not supported");
  mjhipModel hm;
  model_view(m, d, &hm);
  mjhipData hd;
  data_fields(d, &hd);
  mjhip_inverseFD(&hm, &hd, eps, flg_actuation, DfDq, DfDv, DfDa, DsDq, DsDv, DsDa, DmDq);
}

/* mj_rne / mj_xfrcAccumulate on the device, for callers that link them explicitly (the
 * reference's own definitions stay in engine_core_smooth.c / engine_support.c) */
void mj_rne_mjhip(const mjModel* m, mjData* d, int flg_acc, mjtNum* result) {
  mjhipModel hm;
  model_view(m, d, &hm);
  mjhipData hd;
  data_fields(d, &hd);
  mjhip_rne(&hm, &hd, flg_acc, result);
}

void mj_xfrcAccumulate_mjhip(const mjModel* m, mjData* d, mjtNum* qfrc) {
  mjhipModel hm;
  model_view(m, d, &hm);
  mjhipData hd;
  data_fields(d, &hd);
  mjhip_xfrcAccumulate(&hm, &hd, qfrc);
}
