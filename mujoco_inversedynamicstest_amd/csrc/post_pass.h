// post_pass.h — work the generated (straight-line) kernels leave to a pass of their own.
//
// Fluid forces (mj_fluid, engine_passive.c:402-428) read only what the generated kernel has
// stored by the end of its velocity stage (body frames, cvel, geom frames, subtree COM), and
// they enter mj_inverse only through qfrc_passive, which the constraint kernel's final
// assembly reads. So a model with fluid runs its generated kernel (which leaves qfrc_fluid
// zero), then this pass, then the constraint kernel for every instance (codegen's
// constraint_mode 'all'), and every output equals the generic pipeline's: qfrc_passive is
// re-formed here in mj_passive's own order (spring + damper, + fluid, + gravcomp, :461-493).
//
// Spatial tendons (mj_tendon, engine_core_smooth.c:651-860) depend on site and geom frames
// at run time, so the generated kernel leaves their length, Jacobian and velocity, the
// tendon transmissions on them and every tendon term of mj_passive to tendonAfter below,
// which runs before the constraint kernel (constraint_mode 'all'): mj_tendon, the
// ten_velocity of mj_fwdVelocity, those transmissions and all of mj_passive (fluid included)
// are re-formed with the generic functions, over the frames the generated kernel stored.
//
// mjENBL_INVDISCRETE (mj_inverseSkip, engine_inverse.c:197-256): the generated kernel runs
// the position and velocity stages and an RNE over the caller's qacc. discreteBefore then
// saves qacc, replaces it with mj_discreteAcc's (engine_inverse.c:81-164) and redoes
// mj_rne(flg_acc = 1) over it; the constraint kernel (constraint_mode 'all', its rows made
// after the new qacc is in place, fastFusedOk) assembles qfrc_inverse, the
// sensor pass runs mj_sensorAcc on it, and discreteRestore puts the caller's qacc back, as
// the reference does after its sensors. It runs after the tendon or fluid pass: implicit
// damping reads tendon Jacobians and the passive derivatives.
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

MJH_HD bool hasSpatial(const mjhipModel& m) {
  for (int i = 0; i < m.ntendon; i++) {
    if (m.wrap_type[m.tendon_adr[i]] != mjhipWRAP_JOINT) return true;
  }
  return false;
}

template <int S>
MJH_HD void tendonAfter(const mjhipModel& m, const Lane<S>& d) {
  const int nv = m.nv;
  tendon(m, d);                             // fixed tendons re-formed to the same values
  for (int r = 0; r < m.ntendon; r++) d.ten_velocity[r] = dot(d.ten_J + r*nv, d.qvel, nv);
  for (int i = 0; i < m.nu; i++) {          // mj_transmission :1053-1081 on spatial tendons
    if (m.actuator_trntype[i] != mjhipTRN_TENDON) continue;
    const int id = m.actuator_trnid[2*i];
    if (m.wrap_type[m.tendon_adr[id]] == mjhipWRAP_JOINT) continue;
    const int adr = m.moment_rowadr[i];
    const double gear = m.actuator_gear[6*i];
    d.actuator_length[i] = d.ten_length[id]*gear;
    for (int k = 0; k < m.moment_rownnz[i]; k++) {
      d.actuator_moment[adr+k] = d.ten_J[id*nv + m.moment_colind[adr+k]]*gear;
    }
    if (!(m.opt.disableflags & mjhipDSBL_ACTUATION)) {
      d.actuator_velocity[i] = dotSparse(d.actuator_moment + adr, d.qvel, m.moment_rownnz[i],
                                         m.moment_colind + adr);
    }
  }
  passive(m, d);
}

MJH_HD bool hasDiscrete(const mjhipModel& m) {
  return (m.opt.enableflags & mjhipENBL_INVDISCRETE) != 0;
}

// whether the constraint kernel after the generated kernels takes the fused rows. The
// generic pipeline cannot under INVDISCRETE (its rows would be finished before
// mj_discreteAcc), but here the discrete pass has replaced qacc before the constraint kernel
// starts, so the fused rows see the qacc the reference's mj_invConstraint sees.
MJH_HD bool fastFusedOk(const mjhipModel& m) {
  mjhipModel f = m;
  f.opt.enableflags &= ~mjhipENBL_INVDISCRETE;
  return fusedOk(f, mjhipSTAGE_NONE);
}

template <int S>
MJH_HD void discreteBefore(const mjhipModel& m, const Lane<S>& d) {
  copy(d.qacc_save, d.qacc, m.nv);
  discreteAcc(m, d);
  rne(m, d, 1, d.qfrc_inverse);
}

template <int S>
MJH_HD void discreteRestore(const mjhipModel& m, const Lane<S>& d) {
  copy(d.qacc, d.qacc_save, m.nv);
}

}  // namespace mjh

#endif  // MJHIP_POST_PASS_H_
