/* adapter_stub.c — TEST INFRASTRUCTURE ONLY (tests/test_adapter_exec.py).
 *
 * A stand-in for libmjhip.so's single-instance entry points whose compute is the CPU oracle
 * (oracle/mj_oracle.c). It keeps libmjhip's data contract (include/mjhip.h:230-235,
 * :393-401): a call reads the rows and contacts of the stages it skips from the caller's
 * efc_* / con_* buffers, writes the rows its stages make with the counts, and leaves every
 * other field of the mjhipData alone. Linking it under integration/engine_inverse_mjhip.c
 * runs the adapter's own code (model and data views, contact AoS <-> SoA, the arena rebuild)
 * on a machine without a GPU; the product library never contains it.
 */
#include <stdlib.h>

#include "../include/mjhip.h"
#include "../oracle/mj_oracle.h"

/* an orEfc over the caller's row buffers (capacities as given), with d's counts */
static orEfc efc_view(mjhipData* d) {
  orEfc e = {0};
  e.capacity = d->efc_capacity;
  e.nefc = d->nefc;
  e.ne = d->ne;
  e.nf = d->nf;
  e.nl = d->nl;
#define XE(type, name, w, stage) e.name = d->name;
  MJHIP_DATA_EFC
#undef XE
  e.con_capacity = d->con_capacity;
  e.ncon = d->ncon;
#define XC(type, name, w, stage) e.name = d->name;
  MJHIP_DATA_CONTACT
#undef XC
  /* compressed rows of a sparse-mode model */
  e.nJ = d->nJ;
  e.efc_J_rownnz = d->efc_J_rownnz;
  e.efc_J_rowadr = d->efc_J_rowadr;
  e.efc_J_colind = d->efc_J_colind;
  e.efc_JT = d->efc_JT;
  e.efc_JT_rownnz = d->efc_JT_rownnz;
  e.efc_JT_rowadr = d->efc_JT_rowadr;
  e.efc_JT_colind = d->efc_JT_colind;
  return e;
}

static void counts_back(mjhipData* d, const orEfc* e) {
  d->nefc = e->nefc;
  d->ne = e->ne;
  d->nf = e->nf;
  d->nl = e->nl;
  d->ncon = e->ncon;
  d->nJ = e->nJ;
}

int mjhip_modelCapacity(const mjhipModel* m, int* efc_rows, int* contacts) {
  if (!m) return MJHIP_ERR_ARG;
  if (efc_rows) *efc_rows = or_efcCapacity(m);
  if (contacts) {
    int n = or_contactCapacity(m);
    *contacts = n < 0 ? 0 : n;
  }
  return MJHIP_OK;
}

void mjhip_inverseSkip(const mjhipModel* m, mjhipData* d, int skipstage, int skipsensor) {
  orEfc e = efc_view(d);
  or_inverseSkip(m, d, &e, skipstage, skipsensor);
  counts_back(d, &e);
}

void mjhip_inverse(const mjhipModel* m, mjhipData* d) {
  mjhip_inverseSkip(m, d, mjhipSTAGE_NONE, 0);
}

void mjhip_invPosition(const mjhipModel* m, mjhipData* d) {
  orEfc e = efc_view(d);
  e.nefc = e.ne = e.nf = e.nl = e.ncon = 0;
  or_invPosition(m, d, &e);
  counts_back(d, &e);
}

void mjhip_invVelocity(const mjhipModel* m, mjhipData* d) {
  orEfc e = efc_view(d);
  or_invVelocity(m, d, &e);
}

void mjhip_invConstraint(const mjhipModel* m, mjhipData* d) {
  orEfc e = efc_view(d);
  or_invConstraint(m, d, &e);
}

void mjhip_compareFwdInv(const mjhipModel* m, mjhipData* d) {
  orEfc e = efc_view(d);
  or_compareFwdInv(m, d, &e);
}

void mjhip_rne(const mjhipModel* m, mjhipData* d, int flg_acc, mjtNum* result) {
  or_rne(m, d, flg_acc, result);
}

void mjhip_xfrcAccumulate(const mjhipModel* m, mjhipData* d, mjtNum* qfrc) {
  or_xfrcAccumulate(m, d, qfrc);
}

/* mjd_inverseFD keeps its rows in scratch of the model's capacity, as the library does */
void mjhip_inverseFD(const mjhipModel* m, mjhipData* d, mjtNum eps, mjtByte flg_actuation,
                     mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa, mjtNum* DsDq, mjtNum* DsDv,
                     mjtNum* DsDa, mjtNum* DmDq) {
  const int rows = or_efcCapacity(m) + 1, cons = or_contactCapacity(m) + 1;
  mjhipData s = *d;
  char* buf = NULL;
  size_t total = 0;
#define SZ(type, w, n) ((sizeof(type) * (size_t)(w) * (n) + 15) & ~(size_t)7)
#define MJ_M(n) m->n
#define XE(type, name, w, stage) total += SZ(type, w, rows);
  MJHIP_DATA_EFC
#undef XE
#define XC(type, name, w, stage) total += SZ(type, w, cons);
  MJHIP_DATA_CONTACT
#undef XC
  buf = (char*)calloc(1, total);
  char* q = buf;
#define XE(type, name, w, stage) s.name = (type*)q; q += SZ(type, w, rows);
  MJHIP_DATA_EFC
#undef XE
#define XC(type, name, w, stage) s.name = (type*)q; q += SZ(type, w, cons);
  MJHIP_DATA_CONTACT
#undef XC
#undef MJ_M
#undef SZ
  s.efc_capacity = rows;
  s.con_capacity = cons;
  orEfc e = efc_view(&s);
  or_inverseFDEx(m, &s, &e, eps, flg_actuation, DfDq, DfDv, DfDa, DsDq, DsDv, DsDa, DmDq);
  d->status = s.status;
  free(buf);
}
