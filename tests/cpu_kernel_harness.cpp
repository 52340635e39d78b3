// cpu_kernel_harness.cpp — TEST ONLY: compiles the HIP engine's per-lane pipeline
// (mujoco_inversedynamicstest_amd/csrc/engine_device.h) for the host with stride 1, so the
// test suite can check the device code's arithmetic bit-for-bit against the oracle without
// a GPU. This is never part of the product library (libmjhip.so has no CPU path).
#include <stdlib.h>
#include <string.h>

#include "../mujoco_inversedynamicstest_amd/csrc/engine_device.h"
#include "../mujoco_inversedynamicstest_amd/csrc/pair_program.h"

// doubles / ints of per-instance scratch (each field padded by one element)
extern "C" void kh_sizes(const mjhipModel* m, int efc_cap, int con_cap, long* nd, long* ni) {
  const int nv = m->nv, nbody = m->nbody;
  (void)nv; (void)nbody;
  long d = 0, i = 0;
#define XSC(name, n) d += (long)(n) + 1;
  MJHIP_SCRATCH_FIELDS
#undef XSC
#define XSI(name, n) i += (long)(n) + 1;
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
  *nd = d;
  *ni = i;
}

// offset (elements) and length of a scratch field; returns 0 double, 1 int, -1 unknown
extern "C" int kh_field(const mjhipModel* m, int efc_cap, int con_cap, const char* field,
                        long* offset, long* len) {
  const int nv = m->nv, nbody = m->nbody;
  (void)nv; (void)nbody;
  long d = 0, i = 0;
#define XSC(name, n) if (!strcmp(field, #name)) { *offset = d; *len = (n); return 0; } \
  d += (long)(n) + 1;
  MJHIP_SCRATCH_FIELDS
#undef XSC
#define XSI(name, n) if (!strcmp(field, #name)) { *offset = i; *len = (n); return 1; } \
  i += (long)(n) + 1;
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
  return -1;
}

// scratch / iscratch persist between calls, like the device mirror, so skipstage > NONE sees
// the earlier stages' constraint rows and contacts
static mjh::Lane<1> bind(const mjhipModel* m, mjhipData* d, double* scratch, int* iscratch,
                         int efc_cap, int con_cap);

// classic = 1 forces the unfused constraint path; otherwise the path follows the GPU
// dispatch (fused when mjh::fusedOk)
extern "C" int kh_inverse(const mjhipModel* m, mjhipData* d, double* scratch, int* iscratch,
                          int efc_cap, int con_cap, int skipstage, int classic) {
  mjh::Lane<1> L = bind(m, d, scratch, iscratch, efc_cap, con_cap);
  int st = (!classic && mjh::fusedOk(*m, skipstage)) ?
      mjh::inverseSkip<1, true, true>(*m, L, skipstage) : mjh::inverseSkip(*m, L, skipstage);
  d->nefc = L.efc_count[0];
  return st;
}

extern "C" int kh_forward(const mjhipModel* m, mjhipData* d, double* scratch, int* iscratch,
                          int efc_cap, int con_cap) {
  mjh::Lane<1> L = bind(m, d, scratch, iscratch, efc_cap, con_cap);
  int st = mjh::forwardSkip(*m, L, mjhipSTAGE_NONE);
  d->nefc = L.efc_count[0];
  return st;
}

static mjh::Lane<1> bind(const mjhipModel* m, mjhipData* d, double* scratch, int* iscratch,
                         int efc_cap, int con_cap) {
  mjh::Lane<1> L;
#define XD(name, d0, d1, stage) L.name.p = d->name;
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD
#undef XD
  const int nv = m->nv, nbody = m->nbody;
  (void)nv; (void)nbody;
  double* p = scratch;
#define XSC(name, n) L.name.p = p; p += (long)(n) + 1;
  MJHIP_SCRATCH_FIELDS
#undef XSC
  int* q = iscratch;
#define XSI(name, n) L.name.p = q; q += (long)(n) + 1;
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
  // mjData fields that are device scratch: bound to the host data so tests compare them
  L.time.p = &d->time;
  if (mjh_needSubtreeVel(m)) {
    L.subtree_linvel.p = d->subtree_linvel;
    L.subtree_angmom.p = d->subtree_angmom;
  }
  if (mjh_needRnePost(m)) {
    L.cacc.p = d->cacc;
    L.cfrc_int.p = d->cfrc_int;
    L.cfrc_ext.p = d->cfrc_ext;
  }
  L.efc_cap = efc_cap;
  L.con_cap = con_cap;
  L.nj_cap = mjh_njCap(m, efc_cap);
  static unsigned long long chain[64];
  for (int k = 0; k < m->nbody && k < 64; k++) chain[k] = mjh::chainMask(*m, k);
  L.chain = chain;
  L.gxpos = L.geom_xpos;
  L.gstage = false;
  L.cdq = nullptr;
  L.fst = nullptr;
  L.nfst = 0;
  L.cbody = nullptr;
  L.ncbody = 0;
  L.dchain = nullptr;
  L.ccdx = L.ccd.p;
  L.ccdxi = L.ccdi.p;
  // the static collision program, as libmjhip.so builds it per context (rebuilt per call
  // here: the harness keeps no per-model state)
  static std::vector<CoopPair> prog;
  static std::vector<int> ipair;
  const std::vector<ProgItem> items = collision_pairs(m);
  prog = coop_program(m, items);
  ipair.resize(items.size());
  for (size_t k = 0; k < items.size(); k++) ipair[k] = items[k].ipair;
  const bool use = !prog.empty();
  L.prog = use ? prog.data() : nullptr;
  L.prog_ipair = use ? ipair.data() : nullptr;
  L.nprog = use ? (int)prog.size() : 0;
  return L;
}

// mjc_ccd on two geoms at the given frames (mjh::ccdGeneral, the function mjhip_ccdBatch runs
// per pair on the device); out: dist, nx, x1[3*50], x2[3*50]
extern "C" int kh_ccd(const mjhipModel* m, int g1, int g2, const double* pos1,
                      const double* mat1, const double* pos2, const double* mat2,
                      double margin, int N, double tol, int maxc, double cutoff, double* out) {
  std::vector<double> x(mjh::ccdScratchDoubles(N));
  std::vector<int> xi(mjh::ccdScratchInts(N));
  return mjh::ccdGeneral<true>(*m, g1, g2, pos1, mat1, pos2, mat2, margin, N, tol, maxc, cutoff,
                               x.data(), xi.data(), out);
}
