// kern_constraint.hip -- the constraint kernels of the straight-line path: k_constraint (one
// lane per instance) and k_constraint_coop (G lanes per instance), in their own translation
// unit of libmjhip.so (kernels.h).
#define MJHIP_KERNEL_UNIT 1
#include "kernels.h"

// constraint part of mj_inverseSkip after the generated kernels (mjh::constraintOnly), over
// the work-list (LIST) or every instance; grid = ceil(B/64) blocks
template <bool CONTACT, bool FUSED, bool LIST>
__global__ __launch_bounds__(64) void k_constraint(mjhipModel m, Mirror mr, int B,
                                                   const int* __restrict__ worklist,
                                                   const int* __restrict__ count,
                                                   double* __restrict__ qfrc_out,
                                                   int* __restrict__ status) {
  const long n = LIST ? (long)*count : (long)B;
  if ((long)blockIdx.x*64 >= n) return;      // whole block idle (uniform): before the barrier
  MJHIP_CHAIN_TABLE(FUSED)
  const long g = (long)blockIdx.x*64 + threadIdx.x;
  if (LIST || !qfrc_out) {
    if (g >= n) return;
    const long inst = LIST ? worklist[g] : g;
    Lane<64> d = lane_view(mr, (int)(inst >> 6), (int)(inst & 63));
    d.chain = chain;
    MJHIP_GEOM_STAGE(CONTACT, FUSED)
    const int st = mjh::constraintOnly<64, CONTACT, FUSED>(m, d);
    if (status && st) status[inst] |= st;   // after the generated kernels' input checks
    if (qfrc_out) {        // a few scattered work-list instances
      for (int k = 0; k < m.nv; k++) qfrc_out[inst*m.nv + k] = d.qfrc_inverse[k];
    }
    return;
  }
  // every instance with a row-major output: the block's rows go out coalesced through LDS
  // (after the geom copy); lanes past B skip the work but join the copy
  double* qo = g_gstage + ((CONTACT && FUSED) ? 3*m.ngeom*64 : 0);
  if (g < n) {
    Lane<64> d = lane_view(mr, (int)(g >> 6), (int)(g & 63));
    d.chain = chain;
    MJHIP_GEOM_STAGE(CONTACT, FUSED)
    const int st = mjh::constraintOnly<64, CONTACT, FUSED>(m, d);
    if (status && st) status[g] |= st;
    for (int k = 0; k < m.nv; k++) qo[threadIdx.x*m.nv + k] = d.qfrc_inverse[k];
  }
  __syncthreads();
  const long rows = n - (long)blockIdx.x*64 < 64 ? n - (long)blockIdx.x*64 : 64;
  double* dst = qfrc_out + (long)blockIdx.x*64*m.nv;
  for (long r = threadIdx.x; r < rows*m.nv; r += 64) dst[r] = qo[r];
}


// XCD-aware block order: the dispatcher deals workgroups round-robin over the 8 XCDs (block
// b to XCD b % 8), each with its own L2. The logical block returned here numbers the blocks
// an XCD receives consecutively, so the 64 / IPB workgroups of k_constraint_coop that share
// one 64-instance mirror block (a mirror line holds 16 instances' copies of one element) run
// behind one L2 instead of fetching and writing back the same partial lines on eight.
// A bijection on [0, nb) for any nb.
__device__ __forceinline__ long xcdBlock(unsigned b, unsigned nb) {
  constexpr unsigned X = 8;
  const unsigned x = b % X, per = nb / X, rem = nb % X;
  return (long)x*per + (x < rem ? x : rem) + b / X;
}

template <int G, bool CONTACT, bool LIST, bool BOX>
__global__ __launch_bounds__(64) void k_constraint_coop(mjhipModel m, Mirror mr, int B,
                                                        const int* __restrict__ worklist,
                                                        const int* __restrict__ count,
                                                        const CoopPair* __restrict__ pairs,
                                                        const mjh::ContactParam* __restrict__ cparams,
                                                        const unsigned long long* __restrict__ masks,
                                                        int npair,
                                                        double* __restrict__ qfrc_out,
                                                        int* __restrict__ status,
                                                        int* __restrict__ cstat) {
  // cstat non-null: a split launch (mjhip.hip launch_inverse) running beside the fac / va
  // stages: qfrc_constraint and this kernel's status bits (into cstat) only, k_assemble
  // forms qfrc_inverse after both
  constexpr int IPB = 64 / G;               // instances per wave
  const long n = LIST ? (long)*count : (long)B;
  const long bid = xcdBlock(blockIdx.x, gridDim.x);
  if (bid*IPB >= n) return;                 // whole block idle (uniform): before the barriers
  __shared__ unsigned long long chain[64], dchain[64];
  __shared__ long s_inst[64 / G];            // the instance of each group (pooled contact rows)
  __shared__ int s_ntask[64 / G];            // its staged contacts with rows
  // the chain masks (host-built, coop_masks: bodies, then dofs on each body's chain for
  // contactRowsSplit's bit test; the kernel runs for nbody, nv <= 64), the pair program and
  // the geom sizes, once per block, all with independent loads
  if ((int)threadIdx.x < m.nbody) {
    chain[threadIdx.x] = masks[threadIdx.x];
    dchain[threadIdx.x] = masks[m.nbody + threadIdx.x];
  }
  CoopPair* prog = reinterpret_cast<CoopPair*>(g_gstage);
  double* gsize = g_gstage + kCoopPairDoubles*npair;
  if (CONTACT) {
    for (int e = threadIdx.x; e < kCoopPairDoubles*npair; e += 64) {
      g_gstage[e] = reinterpret_cast<const double*>(pairs)[e];
    }
    for (int e = threadIdx.x; e < 3*m.ngeom; e += 64) gsize[e] = m.geom_size[e];
  }
  __syncthreads();
  const int sub = threadIdx.x % G, slot = threadIdx.x / G;
  const int ngeom = m.ngeom;
  // grid-stride over the instances (a work-list launch uses at most one block per SIMD, so
  // an empty or short list costs few workgroups); the bound is uniform over the block
  for (long base = bid*IPB; base < n; base += (long)gridDim.x*IPB) {
  const long g = base + slot;
  const bool active = g < n;                // uniform within a group
  const long inst = active ? (LIST ? (long)worklist[g] : g) : 0;
  Lane<64> d = lane_view(mr, (int)(inst >> 6), (int)(inst & 63));
  d.chain = chain;
  d.dchain = dchain;
  const int nv = m.nv, dsbl = m.opt.disableflags;
  int st = 0, ncon = 0;
  MJH_PHASE0(14, 26);
  // per-instance LDS (dynamic, coopLdsBytes): cdof/qvel/qacc for the contact rows, qpos,
  // the geom frames for the collision phase, its survivor list, and the row forces for
  // J'force; all staged by the group with independent loads
  const int nq = m.nq, per = coopPerInstance(m, npair, d.con_cap, d.efc_cap);
  double* lbase = g_gstage + kCoopPairDoubles*npair + 3*ngeom;
  double* cdq = lbase + (long)slot*per;
  double* qp = cdq + 8*nv;
  double* gx = qp + nq;                     // geom_xpos (3 ngeom)
  double* gm = gx + 3*ngeom;                // geom_xmat (9 ngeom)
  int* surv = reinterpret_cast<int*>(gm + 9*ngeom);
  int* cbody = reinterpret_cast<int*>(gm + 9*ngeom + (npair + 1) / 2);
  const int ncb = coopContacts(d.con_cap);
  int* task = cbody + 4*ncb;                // per staged contact: its first row, its condim
  double* fst = gm + 9*ngeom + (npair + 1) / 2 + 3*ncb;
  // box-box contact positions of this lane's pair (only models with box pairs get the room)
  double* bbuf = lbase + (long)IPB*per + (long)threadIdx.x*kBoxBoxBuf;
  const bool collide = CONTACT && mjhip_contactsEnabled(&m) && npair > 0;
  if (active) {
    for (int e = sub; e < 8*nv; e += G) {
      const int j = e >> 3, c = e & 7;
      cdq[e] = c < 6 ? d.cdof[6*j+c] : (c == 6 ? d.qvel[j] : d.qacc[j]);
    }
    for (int e = sub; e < nq; e += G) qp[e] = d.qpos[e];
    if (collide) {
      for (int e = sub; e < 3*ngeom; e += G) gx[e] = d.geom_xpos[e];
      for (int e = sub; e < 9*ngeom; e += G) gm[e] = d.geom_xmat[e];
    }
  }
  d.cdq = cdq;
  d.fst = fst;
  d.nfst = coopRows(d.efc_cap);
  d.cbody = cbody;
  d.ncbody = ncb;
  __syncthreads();                          // the staged frames visible to the group

  // ---- mj_collision over the static pair program: first mj_filterSphere on every pair
  // (G pairs per round, frames from LDS) into an ordered survivor list, then the
  // narrowphase of the survivors only, G per round
  if (collide) {
    const unsigned long long gmask = G == 64 ? ~0ull : ((1ull << G) - 1) << (slot*G);
    const unsigned long long below = (1ull << (threadIdx.x % 64)) - 1;
    int nsurv = 0;
    for (int p0 = 0; p0 < npair; p0 += G) {
      const int p = p0 + sub;
      bool keep = false;
      if (active && p < npair) {
        const CoopPair& P = prog[p];
        const double* p1 = gx + 3*P.g1;
        const double* p2 = gx + 3*P.g2;
        if (P.filt == 0) {
          const double dif[3] = {p1[0]-p2[0], p1[1]-p2[1], p1[2]-p2[2]};
          keep = !(dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2] > P.bound*P.bound);
        } else if (P.filt <= 2) {           // the plane's normal against the other's centre
          const bool pl1 = P.filt == 1;
          const double* mat = gm + 9*(pl1 ? P.g1 : P.g2);
          const double norm[3] = {mat[2], mat[5], mat[8]};
          double dif[3];
          mjh::sub3(dif, pl1 ? p2 : p1, pl1 ? p1 : p2);
          keep = !(mjh::dot3(dif, norm) > P.bound);
        } else {
          keep = true;
        }
      }
      const unsigned long long bal = __ballot(keep) & gmask;
      if (keep) surv[nsurv + __popcll(bal & below)] = p;
      nsurv += __popcll(bal);
    }
    // rounds over the survivors: the wave runs as many as its busiest group needs
    int rounds = (nsurv + G - 1) / G;
    for (int o = G; o < 64; o <<= 1) rounds = max(rounds, __shfl_xor(rounds, o));
    for (int r = 0; r < rounds; r++) {
      const int s0 = r*G, k = s0 + sub;
      int g1 = 0, g2 = 0, num = 0, cnt = 0, bodies[4] = {0, 0, 0, 0};
      double margin = 0;
      mjh::RawContact raw[2];
      mjh::ContactParam cp{};
      if (active && k < nsurv) {            // narrowphase once: raw contacts kept in registers
        const CoopPair P = prog[surv[k]];
        cp = cparams[surv[k]];              // in flight while the narrowphase computes
        g1 = P.g1;
        g2 = P.g2;
        margin = P.margin;
        bodies[0] = P.b1;
        bodies[1] = P.b2;
        bodies[2] = P.rt1;
        bodies[3] = P.rt2;
        if (P.kmax < 0) {                   // the reference would run a function not built here
          st |= MJHIP_INST_UNSUPPORTED;
        } else if ((P.t1 == mjhipGEOM_PLANE &&
                    (P.t2 == mjhipGEOM_BOX || P.t2 == mjhipGEOM_CYLINDER)) ||
                   (P.t1 == mjhipGEOM_BOX && P.t2 == mjhipGEOM_BOX)) {
          num = -1;                         // plane : box / cylinder, box : box: counts, then stores
          mjh::collidePlaneBoxCyl<64, false, BOX, false>(m, d, g1, g2, margin, cp, cnt, &st,
                                                         bbuf);
        } else {
          num = mjh::narrowPrimitive(P.t1, P.t2, margin, (const double*)(gx + 3*g1),
                                     (const double*)(gm + 9*g1), gsize + 3*g1,
                                     (const double*)(gx + 3*g2), (const double*)(gm + 9*g2),
                                     gsize + 3*g2, raw);
          cnt = num;
        }
      }
      int total;
      const int excl = groupScan<G>(cnt, sub, &total) - cnt;
      if (cnt) {
        int c = ncon + excl;
        if (num < 0) {
          mjh::collidePlaneBoxCyl<64, true, BOX, false>(m, d, g1, g2, margin, cp, c, &st, bbuf);
        } else {
          mjh::storeContacts<64>(m, d, g1, g2, margin, cp, raw, num, c, &st);
        }
        for (int q = ncon + excl; q < c && q < ncb; q++) {   // the contacts just stored
          for (int e = 0; e < 4; e++) cbody[4*q + e] = bodies[e];
        }
      }
      ncon += total;
    }
  }
  if (active && sub == 0) d.con_count[0] = ncon < d.con_cap ? ncon : d.con_cap;
  if (ncon > d.con_cap) ncon = d.con_cap;
  __syncthreads();                          // contacts visible to every lane of the group
  MJH_PHASE(15);

  // ---- mj_makeConstraint: non-contact rows, then contact rows (all finished at creation)
  mjh::RowCount rc;
  if (active && !(dsbl & mjhipDSBL_CONSTRAINT)) {
    if (m.neq) {
      if (sub == 0) mjh::instantiateEquality<64, true>(m, d, rc, &st);
      rc.nefc = __shfl(rc.nefc, 0, G);
      rc.ne = __shfl(rc.ne, 0, G);
    }
    // a non-contact row r: the owner writes J (jval(k) for column k) and finishes it
    auto addRow = [&](auto jval, double pos, double margin, double floss, int tp, int id)
        MJH_LAMBDA_INLINE {
      const int r = rc.nefc;
      if (r + 1 > d.efc_cap) {
        st |= MJHIP_INST_CNSTRFULL;
        return false;
      }
      if (r % G == sub) {
        auto J = d.efc_J + (long)r*nv;
        for (int k = 0; k < nv; k++) J[k] = jval(k);
        rowFields(d, r, pos, margin, floss, tp, id);
        // J*qvel, J*qacc from the row's generator and the LDS copies (the values stored in
        // efc_J, in mju_dot's order), not read back from memory
        const mjh::FnIdx<decltype(jval)> jv{jval};
        mjh::finishNonContactVA(m, d, r, tp, id, pos, margin, floss,
                                mjh::dot(jv, mjh::StridedIdx<8>{cdq + 6}, nv),
                                mjh::dot(jv, mjh::StridedIdx<8>{cdq + 7}, nv));
      }
      rc.nefc++;
      return true;
    };
    // rows of one G-wide round of dofs or joints, placed by a group prefix sum over each
    // lane's row count in the reference's order; a row past the capacity is dropped and
    // flagged, as addRow does
    auto placeRound = [&](int nr, int& counter) MJH_LAMBDA_INLINE {
      int total;
      const int first = rc.nefc + groupScan<G>(nr, sub, &total) - nr;
      const int end = rc.nefc + total < d.efc_cap ? rc.nefc + total : d.efc_cap;
      if (rc.nefc + total > d.efc_cap) st |= MJHIP_INST_CNSTRFULL;
      counter += end - rc.nefc;
      rc.nefc = end;
      return first;
    };
    auto putRow = [&](int r, auto jval, double pos, double margin, double floss, int tp, int id)
        MJH_LAMBDA_INLINE {
      if (r >= d.efc_cap) return;
      auto J = d.efc_J + (long)r*nv;
      for (int k = 0; k < nv; k++) J[k] = jval(k);
      rowFields(d, r, pos, margin, floss, tp, id);
      const mjh::FnIdx<decltype(jval)> jv{jval};
      mjh::finishNonContactVA(m, d, r, tp, id, pos, margin, floss,
                              mjh::dot(jv, mjh::StridedIdx<8>{cdq + 6}, nv),
                              mjh::dot(jv, mjh::StridedIdx<8>{cdq + 7}, nv));
    };
    if (!(dsbl & mjhipDSBL_FRICTIONLOSS)) {
      // dof friction (:785-799), G dofs per round
      for (int i0 = 0; i0 < nv; i0 += G) {
        const int i = i0 + sub;
        const double fl = i < nv ? m.dof_frictionloss[i] : 0.0;
        const int first = placeRound(fl > 0 ? 1 : 0, rc.nf);
        if (fl > 0) {
          putRow(first, [&](int k) { return k == i ? 1.0 : 0.0; }, 0, 0, fl,
                 mjh::CNSTR_FRICTION_DOF, i);
        }
      }
      // tendon friction (:801-815) on the ten_J row; mj_addConstraint drops an empty row
      for (int i = 0; i < m.ntendon; i++) {
        const double fl = m.tendon_frictionloss[i];
        if (!(fl > 0)) continue;
        mjh::SP<64> tj = d.ten_J + (long)i*nv;
        bool nonempty = false;
        for (int k = 0; k < nv && !nonempty; k++) nonempty = tj[k] != 0;
        if (nonempty && addRow([&](int k) { return tj[k]; }, 0, 0, fl,
                               mjh::CNSTR_FRICTION_TENDON, i)) {
          rc.nf++;
        }
      }
    }
    if (!(dsbl & mjhipDSBL_LIMIT)) {
      // joint limits (:824-900), G joints per round: a slide/hinge joint gives up to two
      // rows (lower side first), a ball joint one
      for (int i0 = 0; i0 < m.njnt; i0 += G) {
        const int i = i0 + sub;
        int nr = 0, t = -1, da = 0;
        bool on[2] = {false, false};
        double dist[2] = {0, 0}, aa[3] = {0, 0, 0}, margin = 0;
        if (i < m.njnt && m.jnt_limited[i]) {
          margin = m.jnt_margin[i];
          t = m.jnt_type[i];
          da = m.jnt_dofadr[i];
          if (t == mjhipJNT_SLIDE || t == mjhipJNT_HINGE) {
            const double value = qp[m.jnt_qposadr[i]];
            for (int k = 0; k < 2; k++) {
              const int side = 2*k - 1;
              dist[k] = side * (m.jnt_range[2*i+k] - value);
              on[k] = dist[k] < margin;
              nr += on[k];
            }
          } else if (t == mjhipJNT_BALL) {
            const int adr = m.jnt_qposadr[i];
            double quat[4] = {qp[adr], qp[adr+1], qp[adr+2], qp[adr+3]};
            mjh::normalize4(quat);
            mjh::quat2Vel(aa, quat, 1);
            const double value = mjh::normalize3(aa);
            dist[0] = mjh::dmax(m.jnt_range[2*i], m.jnt_range[2*i+1]) - value;
            on[0] = dist[0] < margin && (aa[0] != 0 || aa[1] != 0 || aa[2] != 0);
            nr = on[0];
          }
        }
        int r = placeRound(nr, rc.nl);
        if (t == mjhipJNT_SLIDE || t == mjhipJNT_HINGE) {
          for (int k = 0; k < 2; k++) {
            if (!on[k]) continue;
            const double sg = -(double)(2*k - 1);
            putRow(r++, [&](int c) { return c == da ? sg : 0.0; }, dist[k], margin, 0,
                   mjh::CNSTR_LIMIT_JOINT, i);
          }
        } else if (t == mjhipJNT_BALL && on[0]) {
          putRow(r, [&](int c) { return (c >= da && c < da + 3) ? aa[c-da]*-1 : 0.0; },
                 dist[0], margin, 0, mjh::CNSTR_LIMIT_JOINT, i);
        }
      }
      for (int i = 0; i < m.ntendon; i++) {
        if (!m.tendon_limited[i]) continue;
        const double value = d.ten_length[i], margin = m.tendon_margin[i];
        mjh::SP<64> tj = d.ten_J + (long)i*nv;
        int nonempty = -1;                  // ten_J row scanned only for an active side
        for (int side = -1; side <= 1; side += 2) {
          const double dist = side * (m.tendon_range[2*i+(side+1)/2] - value);
          if (dist < margin && nonempty < 0) {
            nonempty = 0;
            for (int k = 0; k < nv && !nonempty; k++) nonempty = tj[k] != 0;
          }
          if (dist < margin && nonempty &&
              addRow([&](int k) { return tj[k]*(double)(-side); }, dist, margin, 0,
                     mjh::CNSTR_LIMIT_TENDON, i)) {
            rc.nl++;
          }
        }
      }
    }
    MJH_PHASE(18);
    // contact rows (pyramidal or frictionless: the fused path excludes elliptic cones):
    // kCoopContactLanes lanes per contact (contactRowsSplit), G / kCoopContactLanes contacts
    // per round; a prefix sum over the contacts' row counts (held by each contact's first
    // lane) gives each its first row; wide contacts (condim 4, 6) run on their first lane
    if (CONTACT && !(dsbl & mjhipDSBL_CONTACT) && nv) {
      // the contacts' first rows: a group prefix sum over their row counts, G per round; the
      // first kCoopContacts contacts become tasks for the whole wave (below), the rest (rare)
      // are formed here by the lane that placed them
      int nef = rc.nefc;
      for (int c0 = 0; c0 < ncon; c0 += G) {
        const int c = c0 + sub;
        int rows = 0, dim = 0;
        if (c < ncon && !d.con_exclude[c]) {
          dim = d.con_dim[c];
          rows = dim == 1 ? 1 : 2*(dim - 1);
        }
        int total;
        const int off = nef + groupScan<G>(rows, sub, &total) - rows;
        bool fits = true;
        if (rows && off + rows > d.efc_cap) {   // mjWARN_CNSTRFULL analogue (capacity is exact)
          st |= MJHIP_INST_CNSTRFULL;
          fits = false;
        }
        if (c < ncb && c < ncon) {
          task[2*c] = off;
          task[2*c+1] = fits ? dim : 0;     // 0: no rows
        }
        if (rows && fits) {
          d.con_efc_address[c] = off;
          if (c >= ncb) {
            switch (dim) {
              case 1: mjh::contactRowsFused<64, 1>(m, d, c, off); break;
              case 3: mjh::contactRowsFused<64, 3>(m, d, c, off); break;
              case 4: mjh::contactRowsFused<64, 4>(m, d, c, off); break;
              default: mjh::contactRowsFused<64, 6>(m, d, c, off); break;
            }
          }
        }
        nef += total;
      }
      rc.nefc = nef < d.efc_cap ? nef : d.efc_cap;
    }
  }
  if (sub == 0) {
    s_inst[slot] = inst;
    s_ntask[slot] = (CONTACT && active && !(dsbl & (mjhipDSBL_CONSTRAINT | mjhipDSBL_CONTACT)) &&
                     nv) ? (ncon < ncb ? ncon : ncb) : 0;
  }
  __syncthreads();                          // the tasks and the staged data visible to all

  // ---- contact rows, pooled over the wave: kCoopContactLanes lanes per contact
  // (contactRowsSplit), 64 / kCoopContactLanes contacts per round whichever instance they
  // belong to, so an instance with many contacts does not hold its wave for many rounds
  if (CONTACT) {
    constexpr int Q = kCoopContactLanes;
    int ntot = 0;
    for (int k = 0; k < IPB; k++) ntot += s_ntask[k];
    const int cq = threadIdx.x % Q;
    for (int t0 = 0; t0 < ntot; t0 += 64 / Q) {
      int t = t0 + threadIdx.x / Q, sl = 0;
      while (sl < IPB && t >= s_ntask[sl]) t -= s_ntask[sl++];
      if (sl >= IPB) continue;              // past the wave's tasks (uniform per Q lanes)
      const long ti = s_inst[sl];
      Lane<64> dt = lane_view(mr, (int)(ti >> 6), (int)(ti & 63));
      double* tb = lbase + (long)sl*per;
      int* tcb = reinterpret_cast<int*>(tb + 8*nv + nq + 12*ngeom + (npair + 1) / 2);
      int* ttask = tcb + 4*ncb;
      dt.chain = chain;
      dt.dchain = dchain;
      dt.cdq = tb;
      dt.cbody = tcb;
      dt.ncbody = ncb;
      dt.fst = tb + 8*nv + nq + 12*ngeom + (npair + 1) / 2 + 3*ncb;
      dt.nfst = coopRows(dt.efc_cap);
      const int off = ttask[2*t], dim = ttask[2*t+1];
      switch (dim) {
        case 0: break;
        case 1: mjh::contactRowsSplit<64, 1, Q>(m, dt, t, off, cq); break;
        case 3: mjh::contactRowsSplit<64, 3, Q>(m, dt, t, off, cq); break;
        case 4: if (cq == 0) mjh::contactRowsFused<64, 4>(m, dt, t, off); break;
        default: if (cq == 0) mjh::contactRowsFused<64, 6>(m, dt, t, off); break;
      }
    }
  }
  if (active && sub == 0) {
    d.efc_count[0] = rc.nefc; d.efc_count[1] = rc.ne; d.efc_count[2] = rc.nf;
    d.efc_count[3] = rc.nl;
  }
  __syncthreads();                          // rows and forces visible to every lane
  MJH_PHASE(16);

  // ---- qfrc_constraint = J'force (column-parallel, two columns per lane per pass, eight
  // rows' loads in flight; forces from LDS) and the mj_inverse assembly
  if (active) {
    const int nefc = rc.nefc;
    for (int j0 = sub; j0 < nv; j0 += 2*G) {
      const int j1 = j0 + G;
      const bool has1 = j1 < nv;
      // the assembly's inputs, loaded ahead of the rows (a load issued after this lane's
      // stores would wait for them); a split launch assembles in k_assemble
      const bool asmb = !cstat;
      const double rne0 = asmb ? (double)d.qfrc_inverse[j0] : 0.0, arm0 = m.dof_armature[j0];
      const double pas0 = asmb ? (double)d.qfrc_passive[j0] : 0.0, qa0 = cdq[8*j0 + 7];
      const double rne1 = (asmb && has1) ? (double)d.qfrc_inverse[j1] : 0.0;
      const double arm1 = has1 ? m.dof_armature[j1] : 0.0;
      const double pas1 = (asmb && has1) ? (double)d.qfrc_passive[j1] : 0.0;
      const double qa1 = has1 ? cdq[8*j1 + 7] : 0.0;
      double acc0 = 0, acc1 = 0;
      for (int r0 = 0; r0 < nefc; r0 += 8) {
        double f[8], x0[8], x1[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int r = r0 + u;
          f[u] = r < nefc ? (r < d.nfst ? fst[r] : d.efc_force[r]) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
          auto Jr = d.efc_J + (long)(r0 + u)*nv;
          x0[u] = f[u] != 0 ? Jr[j0] : 0.0;
          x1[u] = (f[u] != 0 && has1) ? Jr[j1] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {   // mju_mulMatTVec's row order, zero forces skipped
          if (f[u] != 0) {
            acc0 += x0[u]*f[u];
            acc1 += x1[u]*f[u];
          }
        }
      }
      d.qfrc_constraint[j0] = acc0;
      if (has1) d.qfrc_constraint[j1] = acc1;
      if (!asmb) continue;
      const double out0 = rne0 + (arm0 * qa0 - pas0 - acc0);
      d.qfrc_inverse[j0] = out0;
      if (qfrc_out) qfrc_out[inst*nv + j0] = out0;
      if (has1) {
        const double out1 = rne1 + (arm1 * qa1 - pas1 - acc1);
        d.qfrc_inverse[j1] = out1;
        if (qfrc_out) qfrc_out[inst*nv + j1] = out1;
      }
    }
    for (int o = G/2; o; o >>= 1) st |= __shfl_xor(st, o, G);
    if (sub == 0 && cstat) cstat[inst] = st;
    else if (sub == 0 && status && st) status[inst] |= st;
  }
  MJH_PHASE(17);
  __syncthreads();                          // the group's LDS is reused by the next round
  }
}

template __global__ void k_constraint<true, true, false>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
template __global__ void k_constraint<true, false, false>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
template __global__ void k_constraint<false, true, false>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
template __global__ void k_constraint<false, false, false>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
template __global__ void k_constraint<false, true, true>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
template __global__ void k_constraint<false, false, true>(mjhipModel, Mirror, int, const int*, const int*, double*, int*);
template __global__ void k_constraint_coop<16, true, true, true>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
template __global__ void k_constraint_coop<16, true, false, true>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
template __global__ void k_constraint_coop<16, true, true, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
template __global__ void k_constraint_coop<16, true, false, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
template __global__ void k_constraint_coop<16, false, true, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
template __global__ void k_constraint_coop<16, false, false, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
// lane-count variants of the contact path (MJHIP_COOP_LANES=8 / 32, measurement only)
template __global__ void k_constraint_coop<8, true, false, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);
template __global__ void k_constraint_coop<32, true, false, false>(mjhipModel, Mirror, int, const int*, const int*, const CoopPair*, const mjh::ContactParam*, const unsigned long long*, int, double*, int*, int*);

MJHIP_TIMER_SETTER(mjhip_setTimerBufConstraint)
