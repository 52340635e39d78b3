// post_pass.h — work the generated (straight-line) kernels leave to a pass of their own.
//
// Fluid forces (mj_fluid, engine_passive.c:402-428) read only what the generated kernel has
// stored by the end of its velocity stage (body frames, cvel, geom frames, subtree COM), and
// they enter mj_inverse only through qfrc_passive, which the constraint kernel's final
// assembly reads. So a model with fluid runs its generated kernel (which leaves qfrc_fluid
// zero), then this pass, then the constraint kernel for every instance (codegen's
// constraint_mode 'all'), and every output equals the generic pipeline's: qfrc_passive is
// re-formed here in mj_passive's own order (spring + damper, + fluid, + gravcomp, :461-493).
#ifndef MJHIP_POST_PASS_H_
#define MJHIP_POST_PASS_H_

#include "engine_device.h"

namespace mjh {

MJH_HD bool hasFluid(const mjhipModel& m) {
  return !(m.opt.disableflags & mjhipDSBL_PASSIVE) && (m.opt.viscosity > 0 || m.opt.density > 0);
}

template <int S>
MJH_HD void fluidAfter(const mjhipModel& m, const Lane<S>& d) {
  if (!hasFluid(m)) return;
  const int nv = m.nv;
  zero(d.qfrc_fluid, nv);
  for (int i = 1; i < m.nbody; i++) {       // the ellipsoid model where a geom asks for it
    if (m.body_mass[i] < MINVAL) continue;
    int ell = 0;
    for (int j = 0; j < m.body_geomnum[i] && ell == 0; j++) {
      ell += m.geom_fluid[12*(m.body_geomadr[i] + j)] > 0;
    }
    if (ell) ellipsoidFluid(m, d, i);
    else inertiaBoxFluid(m, d, i);
  }
  add(d.qfrc_passive, d.qfrc_spring, d.qfrc_damper, nv);
  addTo(d.qfrc_passive, d.qfrc_fluid, nv);
  const double* g = m.opt.gravity;
  bool gravcomp = false;
  if (m.ngravcomp && !(m.opt.disableflags & mjhipDSBL_GRAVITY) &&
      sqrt(g[0]*g[0] + g[1]*g[1] + g[2]*g[2]) != 0) {
    for (int i = 1; i < m.nbody; i++) gravcomp = gravcomp || m.body_gravcomp[i] != 0;
  }
  if (gravcomp) {
    for (int i = 0; i < m.njnt; i++) {
      if (m.jnt_actgravcomp[i]) continue;
      const int t = m.jnt_type[i];
      const int dofnum = t == mjhipJNT_FREE ? 6 : (t == mjhipJNT_BALL ? 3 : 1);
      const int dofadr = m.jnt_dofadr[i];
      for (int j = 0; j < dofnum; j++) d.qfrc_passive[dofadr+j] += d.qfrc_gravcomp[dofadr+j];
    }
  }
}

}  // namespace mjh

#endif  // MJHIP_POST_PASS_H_
