/* adapter_harness.c — TEST INFRASTRUCTURE ONLY (tests/test_adapter_exec.py).
 *
 * Runs the reference-side adapter integration/engine_inverse_mjhip.c on real mjModel /
 * mjData structs laid out by the reference's public headers (include/mujoco/mjmodel.h,
 * mjdata.h), without the reference's library:
 *   - the mjhip_* calls resolve to tests/adapter_stub.c (the CPU oracle behind libmjhip's
 *     data contract);
 *   - the three engine symbols the adapter calls are defined here: mj_arenaAllocByte
 *     (engine_io.c:1563-1606, without the ASan/thread-pool branches), mj_warning
 *     (engine_support.c:1650-1667, the counter part) and mju_error (engine_util_errmem.c:
 *     118-150; here it records the message and unwinds to the caller of hx_call).
 * The mjModel is a view of a compiled mjhipModel (pointer copies: the adapter's own
 * model_view() is the inverse mapping) and the mjData owns its arrays and a real arena.
 */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mujoco/mujoco.h>
#include <mujoco/mjxmacro.h>

#include "mjhip.h"

void* mj_arenaAllocByte(mjData* d, size_t bytes, size_t alignment);

static jmp_buf g_jmp;
static int g_in_call = 0;
static char g_err[1024];

void mju_error(const char* msg, ...) {
  va_list ap;
  va_start(ap, msg);
  vsnprintf(g_err, sizeof(g_err), msg, ap);
  va_end(ap);
  if (g_in_call) longjmp(g_jmp, 1);
  fprintf(stderr, "mju_error outside hx_call: %s\n", g_err);
  abort();
}

void mj_warning(mjData* d, int warning, int info) {
  d->warning[warning].lastinfo = info;
  d->warning[warning].number++;
}

void* mj_arenaAllocByte(mjData* d, size_t bytes, size_t alignment) {
  size_t misalignment = d->parena % alignment;
  size_t padding = misalignment ? alignment - misalignment : 0;
  if (d->parena + padding + bytes > d->narena - d->pstack) return NULL;
  void* result = (char*)d->arena + d->parena + padding;
  d->parena += padding + bytes;
  if (d->pstack + d->parena > d->maxuse_arena) d->maxuse_arena = d->pstack + d->parena;
  return result;
}

typedef struct {
  mjModel* m;
  mjData* d;
} HX;

HX* hx_create(const mjhipModel* hm, long narena) {
  HX* h = (HX*)calloc(1, sizeof(HX));
  mjModel* m = h->m = (mjModel*)calloc(1, sizeof(mjModel));
#define XS(name) m->name = hm->name;
  MJHIP_MODEL_SIZES
#undef XS
  m->opt.timestep = hm->opt.timestep;
  m->opt.impratio = hm->opt.impratio;
  memcpy(m->opt.gravity, hm->opt.gravity, sizeof(m->opt.gravity));
  memcpy(m->opt.wind, hm->opt.wind, sizeof(m->opt.wind));
  memcpy(m->opt.magnetic, hm->opt.magnetic, sizeof(m->opt.magnetic));
  m->opt.density = hm->opt.density;
  m->opt.viscosity = hm->opt.viscosity;
  m->opt.o_margin = hm->opt.o_margin;
  memcpy(m->opt.o_solref, hm->opt.o_solref, sizeof(m->opt.o_solref));
  memcpy(m->opt.o_solimp, hm->opt.o_solimp, sizeof(m->opt.o_solimp));
  memcpy(m->opt.o_friction, hm->opt.o_friction, sizeof(m->opt.o_friction));
  m->opt.ccd_tolerance = hm->opt.ccd_tolerance;
  m->opt.ccd_iterations = hm->opt.ccd_iterations;
  m->opt.integrator = hm->opt.integrator;
  m->opt.cone = hm->opt.cone;
  m->opt.jacobian = hm->opt.jacobian;
  m->opt.disableflags = hm->opt.disableflags;
  m->opt.enableflags = hm->opt.enableflags;
#define X(type, name, d0, d1) m->name = hm->name;
  MJHIP_MODEL_POINTERS_M
#undef X
  m->nconmax = -1;   /* the compiler defaults (mjmodel.h: -1 = no limit but the arena) */
  m->njmax = -1;

  mjData* d = h->d = (mjData*)calloc(1, sizeof(mjData));
#undef MJ_M
#define MJ_M(n) hm->n
#define XD(name, d0, d1, stage) d->name = (mjtNum*)calloc((size_t)(hm->d0) * (d1) + 1, sizeof(mjtNum));
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
  MJHIP_DATA_SENSOR_AUX
#undef XD
#undef MJ_M
#define MJ_M(n) n
#define X(type, name, d0, d1) d->name = hm->name;
  MJHIP_MODEL_POINTERS_D
#undef X
  /* ten_J's compressed structure (mjData, used by sparse-mode models) */
  d->ten_J_rownnz = (int*)calloc((size_t)hm->ntendon + 1, sizeof(int));
  d->ten_J_rowadr = (int*)calloc((size_t)hm->ntendon + 1, sizeof(int));
  d->ten_J_colind = (int*)calloc((size_t)hm->ntendon * hm->nv + 1, sizeof(int));
  memcpy(d->qpos, hm->qpos0, sizeof(mjtNum) * hm->nq);
  d->narena = (size_t)narena;
  d->arena = aligned_alloc(64, ((size_t)narena + 63) & ~(size_t)63);
  memset(d->arena, 0, (size_t)narena);
  d->contact = (mjContact*)d->arena;
  return h;
}

void hx_free(HX* h) {
  mjData* d = h->d;
#define XD(name, d0, d1, stage) free(d->name);
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
  MJHIP_DATA_SENSOR_AUX
#undef XD
  free(d->ten_J_rownnz);
  free(d->ten_J_rowadr);
  free(d->ten_J_colind);
  free(d->arena);
  free(d);
  free(h->m);
  free(h);
}

/* the adapter's entry points; returns 0, or 1 when mju_error was raised (hx_error) */
int hx_call(HX* h, int which, int skipstage, int skipsensor) {
  g_err[0] = 0;
  g_in_call = 1;
  if (setjmp(g_jmp)) {
    g_in_call = 0;
    return 1;
  }
  switch (which) {
    case 0: mj_inverseSkip(h->m, h->d, skipstage, skipsensor); break;
    case 1: mj_inverse(h->m, h->d); break;
    case 2: mj_invPosition(h->m, h->d); break;
    case 3: mj_invVelocity(h->m, h->d); break;
    case 4: mj_invConstraint(h->m, h->d); break;
    case 5: mj_compareFwdInv(h->m, h->d); break;
  }
  g_in_call = 0;
  return 0;
}

const char* hx_error(void) { return g_err; }

/* a data field (MJHIP_DATA_* name) or an arena pointer (MJDATA_ARENA_POINTERS name) */
void* hx_field(HX* h, const char* name) {
  mjData* d = h->d;
#define XD(n, d0, d1, stage) if (!strcmp(name, #n)) return d->n;
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
  MJHIP_DATA_SENSOR_AUX
#undef XD
#define X(type, n, nr, nc) if (!strcmp(name, #n)) return (void*)d->n;
  MJDATA_ARENA_POINTERS
#undef X
  if (!strcmp(name, "arena")) return d->arena;
  if (!strcmp(name, "ten_J_rownnz")) return d->ten_J_rownnz;
  if (!strcmp(name, "ten_J_rowadr")) return d->ten_J_rowadr;
  if (!strcmp(name, "ten_J_colind")) return d->ten_J_colind;
  return NULL;
}

/* byte offset of an arena array from the arena start, -1 when the pointer is NULL, -2 when
 * the name is unknown */
long hx_arena_offset(HX* h, const char* name) {
  mjData* d = h->d;
#define X(type, n, nr, nc) \
  if (!strcmp(name, #n)) return d->n ? (long)((char*)d->n - (char*)d->arena) : -1;
  MJDATA_ARENA_POINTERS
#undef X
  return -2;
}

/* an MJDATA_SCALAR field (size_t, int; time as its integer part) */
long long hx_scalar(HX* h, const char* name) {
  mjData* d = h->d;
#define X(type, n) if (!strcmp(name, #n)) return (long long)d->n;
  MJDATA_SCALAR
#undef X
  return -1;
}

void hx_set_scalar(HX* h, const char* name, long long v) {
  mjData* d = h->d;
#define X(type, n) if (!strcmp(name, #n)) d->n = (type)v;
  MJDATA_SCALAR
#undef X
}

int hx_warning(HX* h, int w) { return h->d->warning[w].number; }
int hx_warning_info(HX* h, int w) { return h->d->warning[w].lastinfo; }

void hx_set_model_int(HX* h, const char* name, int v) {
  if (!strcmp(name, "npair")) h->m->npair = v;
  if (!strcmp(name, "nflex")) h->m->nflex = v;
  if (!strcmp(name, "nplugin")) h->m->nplugin = v;
}

double* hx_solver_fwdinv(HX* h) { return h->d->solver_fwdinv; }

long hx_sizeof_contact(void) { return (long)sizeof(mjContact); }

/* contact i of d->contact: 29 doubles (dist, pos, frame, includemargin, friction, solref,
 * solreffriction, solimp, mu) and 13 ints (dim, geom[2], exclude, efc_address, geom1, geom2,
 * flex[2], elem[2], vert[2]) */
void hx_contact(HX* h, int i, double* dv, int* iv) {
  const mjContact* c = h->d->contact + i;
  double* p = dv;
  *p++ = c->dist;
  for (int k = 0; k < 3; k++) *p++ = c->pos[k];
  for (int k = 0; k < 9; k++) *p++ = c->frame[k];
  *p++ = c->includemargin;
  for (int k = 0; k < 5; k++) *p++ = c->friction[k];
  for (int k = 0; k < 2; k++) *p++ = c->solref[k];
  for (int k = 0; k < 2; k++) *p++ = c->solreffriction[k];
  for (int k = 0; k < 5; k++) *p++ = c->solimp[k];
  *p++ = c->mu;
  int* q = iv;
  *q++ = c->dim;
  *q++ = c->geom[0];
  *q++ = c->geom[1];
  *q++ = c->exclude;
  *q++ = c->efc_address;
  *q++ = c->geom1;
  *q++ = c->geom2;
  *q++ = c->flex[0];
  *q++ = c->flex[1];
  *q++ = c->elem[0];
  *q++ = c->elem[1];
  *q++ = c->vert[0];
  *q++ = c->vert[1];
}
