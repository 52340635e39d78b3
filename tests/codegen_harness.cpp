// codegen_harness.cpp — TEST ONLY: host build of a generated straight-line body
// (codegen.py) plus the generic pipeline for its work-list, over a host mirror, so the test
// suite can check the generated code bit-for-bit against the oracle without a GPU.
#include <stdlib.h>
#include <string.h>

#include "../mujoco_inversedynamicstest_amd/csrc/engine_device.h"
#include "../mujoco_inversedynamicstest_amd/csrc/post_pass.h"
#include "../mujoco_inversedynamicstest_amd/csrc/pair_program.h"
#include GEN_INC

template <bool C, bool F>
static void constraint_part(const mjhipModel* m, Mirror& mr, int inst) {
  static unsigned long long chain[64];
  for (int k = 0; k < m->nbody && k < 64; k++) chain[k] = mjh::chainMask(*m, k);
  mjh::Lane<64> d = lane_view(mr, inst / 64, inst % 64);
  d.chain = chain;
  mjh::constraintOnly<64, C, F>(*m, d);
}

// mjd_inverseFD's store elision (Mirror::fd_elide, codegen.FD_KEEP): instance blocks from
// full_blk on drop their elided stores; -1 (the default) stores everything
static int g_full_blk = -1;
extern "C" void cg_set_full_blk(int full_blk) { g_full_blk = full_blk; }

// fields: concatenated per-instance outputs, row-major [field][inst][k] in MJHIP_DATA_FIELDS
// order. cmode as codegen.constraint_mode (0 none, 1 work-list, 2 all): the constraint
// kernel's part runs on the served instances, as launch_inverse does on the device. Returns
// the number of served instances.
extern "C" int cg_run(const mjhipModel* m, int B, const double* qpos, const double* qvel,
                      const double* qacc, double* out, int efc_cap, int con_cap, int cmode) {
  const int nblk = (B + 63) / 64;
  Mirror mr;
  memset(&mr, 0, sizeof(mr));
  const int nv = m->nv, nbody = m->nbody;
  (void)nv; (void)nbody; (void)con_cap;
#define MJ_M(n) m->n
  int maxs = 1;
#define XD(name, d0, d1, stage) mr.name##_n = (m->d0) * (d1); \
  maxs = mr.name##_n > maxs ? mr.name##_n : maxs; \
  mr.name = (double*)calloc((size_t)nblk * 64 * (mr.name##_n + 1), sizeof(double));
  MJHIP_DATA_FIELDS
  MJHIP_DATA_FORWARD              /* zero inputs the sensor pass reads (xfrc_applied, ...) */
#undef XD
#define XSC(name, n) mr.name##_n = (n); \
  mr.name = (double*)calloc((size_t)nblk * 64 * ((n) + 1), sizeof(double));
  MJHIP_SCRATCH_FIELDS
#undef XSC
#define XSI(name, n) mr.name##_n = (n); \
  mr.name = (int*)calloc((size_t)nblk * 64 * ((n) + 1), sizeof(int));
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
  (void)maxs;
  if (g_full_blk >= 0) {
    mr.fd_elide = 1;
    mr.full_blk = g_full_blk;
  }
  mr.efc_cap = efc_cap;
  mr.con_cap = con_cap;
  mr.nj_cap = mjh_njCap(m, efc_cap);
  // the static collision program, as libmjhip.so builds it per context
  const std::vector<ProgItem> items = collision_pairs(m);
  std::vector<CoopPair> prog = coop_program(m, items);
  std::vector<int> ipair(items.size());
  for (size_t k = 0; k < items.size(); k++) ipair[k] = items[k].ipair;
  mr.prog = prog.empty() ? nullptr : prog.data();
  mr.prog_ipair = prog.empty() ? nullptr : ipair.data();
  mr.nprog = (int)prog.size();
  int* wl = (int*)calloc(B + 1, sizeof(int));
  int wc = 0, wnext = 1;
  for (int i = 0; i < B; i++) {
    FAST_BODY(mr, i / 64, i % 64, B, qpos, qvel, qacc, nullptr, nullptr, wl, &wc, &wnext,
              mr.efc_count);
  }
  const bool spatial = mjh::hasSpatial(*m);
  for (int i = 0; i < B; i++) {   // k_tendon_after, else k_fluid_after, on the device
    mjh::Lane<64> d = lane_view(mr, i / 64, i % 64);
    if (spatial) mjh::tendonAfter<64>(*m, d);
    else mjh::fluidAfter<64>(*m, d);
    if (mjh::hasDiscrete(*m)) {                                  // k_discrete_before
      if (mjh_needTrnAfter(m)) mjh::transmissionAfter<64>(*m, d);
      mjh::discreteBefore<64>(*m, d);
    }
  }
  const bool fused = mjh::fastFusedOk(*m);
  const int served = cmode == 2 ? B : (cmode == 1 ? wc : 0);
  for (int g = 0; g < served; g++) {
    const int inst = cmode == 2 ? g : wl[g];
    if (con_cap > 0) {
      if (fused) constraint_part<true, true>(m, mr, inst);
      else constraint_part<true, false>(m, mr, inst);
    } else {
      if (fused) constraint_part<false, true>(m, mr, inst);
      else constraint_part<false, false>(m, mr, inst);
    }
  }
  for (int i = 0; i < B; i++) {   // transmission/sensor/energy pass (k_sensors on the device)
    mjh::Lane<64> d = lane_view(mr, i / 64, i % 64);
    mjh::sensorsAfter<64>(*m, d, true, mjh_needTrnAfter(m) && !mjh::hasDiscrete(*m));
    if (mjh::hasDiscrete(*m)) mjh::discreteRestore<64>(*m, d);  // k_discrete_restore
  }
  size_t off = 0;
#define XD(name, d0, d1, stage) { int S = mr.name##_n; \
  for (int i = 0; i < B; i++) for (int k = 0; k < S; k++) \
    out[off + (size_t)i*S + k] = mr.name[((size_t)(i/64)*S + k)*64 + (i%64)]; \
  off += (size_t)B*S; free(mr.name); }
  MJHIP_DATA_FIELDS
#undef XD
#define XD(name, d0, d1, stage) free(mr.name);
  MJHIP_DATA_FORWARD
#undef XD
#undef MJ_M
#define XSC(name, n) free(mr.name);
  MJHIP_SCRATCH_FIELDS
#undef XSC
#define XSI(name, n) free(mr.name);
  MJHIP_SCRATCH_INT_FIELDS
#undef XSI
  free(wl);
  return served;
}
