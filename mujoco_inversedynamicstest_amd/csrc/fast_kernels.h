// fast_kernels.h — the registry entry of a straight-line (model-specialized) kernel, shared by
// mjhip.hip and gen_fast.hip (the bundled models' kernels, a translation unit of their own so
// the two compile in parallel).
#ifndef MJHIP_FAST_KERNELS_H_
#define MJHIP_FAST_KERNELS_H_

#include <hip/hip_runtime.h>

#include "engine_device.h"

struct FastKernelEntry {
  unsigned long long sig;
  void (*launch)(dim3, dim3, hipStream_t, const Mirror&, int, const double*, const double*,
                 const double*, double*, int*, int*, int*, int*, int*,
                 const int* /* device-side instance range {first, end}, or null */);
  const char* name;
  int cmode;   // codegen.constraint_mode: 0 none, 1 work-list, 2 every instance
  // mj_inverseSkip(mjSTAGE_POS) for mjd_inverseFD's qvel/qacc perturbations: the va stage of
  // instances [off, B), position-stage inputs from centre (t - off)/per*sstride (codegen.py
  // k_vaskip); null for run-time kernels and models whose rows serve every instance
  // (the last argument is eps: each skip instance reads its centre's qpos/qvel/qacc and adds
  // eps to the component it perturbs, so k_fd_expand writes only the position-stage block)
  void (*launch_vaskip)(hipStream_t, const Mirror&, int, int, int, int, int*, int*, double);
  // mjd_inverseFD layout 2 in one launch over [off, B) (k_fdskip): the first half of the
  // instances qacc perturbations, mj_inverseSkip(mjSTAGE_VEL), the acceleration stage alone
  // over the centre's position- and velocity-stage outputs; the second half qvel
  // perturbations, mjSTAGE_POS, as k_vaskip (centres (t - off)/per*sstride within each half)
  void (*launch_fdskip)(hipStream_t, const Mirror&, int, int, int, int, int*, int*, double);
  // batched mj_inverseSkip(skipstage) for skipstage POS (k_va) or VEL (k_acc) over [0, B)
  // (qfrc_out row-major or null, status or null, efc_count)
  void (*launch_skip)(hipStream_t, const Mirror&, int, int, double*, int*, int*);
  // models whose rows serve every instance (contacts): the straight-line pipeline in two
  // launches, part 0 the position stage (k_spos), part 1 the fac and va stages (k_sfv), so
  // that the cooperative constraint kernel runs beside part 1 on a second stream (arguments:
  // B, part, qpos/qvel/qacc row-major inputs or null, status, worklist_next, efc_count)
  void (*launch_split)(hipStream_t, const Mirror&, int, int, const double*, const double*,
                       const double*, int*, int*, int*);
  // mjd_inverseFD layout 1 in one launch (k_fdall): the position-stage instances [0, A) and
  // the 2nv skip perturbations per base state after them, each skip wave waiting for its
  // centres' flags (arguments: A, ninst, 2nv, eps, worklist, its counter, the next counter,
  // efc_count, fdflag, the flags, the epoch); null where there is no k_vaskip
  void (*launch_fdall)(hipStream_t, const Mirror&, int, int, int, double, int*, int*, int*,
                       int*, int*, int*, int);
};

// the bundled models' kernels (gen_fast.hip), terminated by an entry with launch = nullptr
const FastKernelEntry* mjhip_fastKernels();
int mjhip_genSetTimerBuf(unsigned long long* p);   // gen_fast.hip's mjh_tbuf
int mjhip_genExactSetTimerBuf(unsigned long long* p);   // gen_fast_exact.hip's

#endif  // MJHIP_FAST_KERNELS_H_
