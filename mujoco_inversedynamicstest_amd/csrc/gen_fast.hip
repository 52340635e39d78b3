// gen_fast.hip — the straight-line mj_inverse kernels of the bundled models (gen_fast.inc,
// written by codegen.py in build()), compiled as their own translation unit and linked into
// libmjhip.so with mjhip.hip.
#include "fast_kernels.h"

#if __has_include("gen_fast.inc")
#include "gen_fast.inc"
#else
static const FastKernelEntry g_fast_kernels[] = {{0ull, nullptr, nullptr, 0, nullptr, nullptr,
                                                  nullptr}};
#endif

const FastKernelEntry* mjhip_fastKernels() { return g_fast_kernels; }

// this translation unit's copy of the per-stage timer pointer (engine_device.h mjh_tbuf;
// mjhip_contextTimers); a blocking copy: timed calls are synchronous
int mjhip_genSetTimerBuf(unsigned long long* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(mjh_tbuf), &p, sizeof(p)) != hipSuccess;
}
