/* engine_inverse_mjhip.c — reference-side adapter: replaces src/engine/engine_inverse.c of
 * fancifulland2718/mujoco_InverseDynamicsTest (MuJoCo 3.3.1) so that mj_inverse,
 * mj_inverseSkip, mj_invPosition, mj_invVelocity, mj_invConstraint and mj_compareFwdInv run
 * on the MI355X through libmjhip.so (include/mjhip.h).
 *
 * mjhipModel/mjhipData use the reference's field names, element types and row-major
 * shapes, so the views below are plain pointer copies generated from the same X-macro
 * tables (include/mjhip_fields.h); a name or type mismatch with mjModel/mjData is a
 * compile error (tests/test_integration.py compiles this file against the reference's
 * public headers).
 *
 * Build (in the reference tree): drop engine_inverse.c from src/engine/CMakeLists.txt,
 * add this file, add <repo>/include to the include path and link libmjhip.so.
 */
#include <stdlib.h>
#include <string.h>

#include <mujoco/mujoco.h>

#include "mjhip.h"

/* one persistent view per mjModel: libmjhip caches its device context by view address */
typedef struct {
  const mjModel* m;
  mjhipModel hm;
} ModelView;

static ModelView g_views[16];
static int g_nviews = 0;

static const mjhipModel* model_view(const mjModel* m, const mjData* d) {
  for (int i = 0; i < g_nviews; i++) {
    if (g_views[i].m == m) return &g_views[i].hm;
  }
  ModelView* v = &g_views[g_nviews < 16 ? g_nviews++ : 15];
  mjhipModel* hm = &v->hm;
  memset(hm, 0, sizeof(*hm));
  v->m = m;
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
  return hm;
}

static void data_view(mjData* d, mjhipData* hd) {
  memset(hd, 0, sizeof(*hd));
  memcpy(hd->energy, d->energy, sizeof(hd->energy));
#define XD(name, d0, d1, stage) hd->name = d->name;
  MJHIP_DATA_FIELDS
#undef XD
#define XD(name, d0, d1, stage) hd->name = d->name;
  MJHIP_DATA_FORWARD
#undef XD
}

void mj_inverseSkip(const mjModel* m, mjData* d, int skipstage, int skipsensor) {
  mjhipData hd;
  data_view(d, &hd);
  mjhip_inverseSkip(model_view(m, d), &hd, skipstage, skipsensor);
  d->solver_fwdinv[0] = hd.solver_fwdinv[0];
  d->solver_fwdinv[1] = hd.solver_fwdinv[1];
  memcpy(d->energy, hd.energy, sizeof(d->energy));
}

void mj_inverse(const mjModel* m, mjData* d) {
  mj_inverseSkip(m, d, mjSTAGE_NONE, 0);
}

void mj_invPosition(const mjModel* m, mjData* d) {
  mjhipData hd;
  data_view(d, &hd);
  mjhip_invPosition(model_view(m, d), &hd);
}

void mj_invVelocity(const mjModel* m, mjData* d) {
  mjhipData hd;
  data_view(d, &hd);
  mjhip_invVelocity(model_view(m, d), &hd);
}

void mj_invConstraint(const mjModel* m, mjData* d) {
  mjhipData hd;
  data_view(d, &hd);
  mjhip_invConstraint(model_view(m, d), &hd);
}

void mj_compareFwdInv(const mjModel* m, mjData* d) {
  mjhipData hd;
  data_view(d, &hd);
  hd.nefc = d->nefc;
  mjhip_compareFwdInv(model_view(m, d), &hd);
  d->solver_fwdinv[0] = hd.solver_fwdinv[0];
  d->solver_fwdinv[1] = hd.solver_fwdinv[1];
}
