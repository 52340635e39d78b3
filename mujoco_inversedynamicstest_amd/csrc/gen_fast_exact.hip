// gen_fast_exact.hip — the straight-line mj_inverse kernels of the bundled models with
// native-solver pairs (gen_fast_exact.inc, written by codegen.generate_registries in build()).
// Compiled without multiply-add contraction throughout (__graft_entry__.UNIT_FLAGS), so these
// models round every operation as the oracle does; their registry entries are in gen_fast.hip.
#include "fast_kernels.h"

#if __has_include("gen_fast_exact.inc")
#include "gen_fast_exact.inc"
#endif

// this translation unit's copy of the per-stage timer pointer (engine_device.h mjh_tbuf)
int mjhip_genExactSetTimerBuf(unsigned long long* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(mjh_tbuf), &p, sizeof(p)) != hipSuccess;
}
