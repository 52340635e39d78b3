// pair_program.h -- the static collision program (host code, shared by libmjhip.so and the
// host build of the device code in tests/cpu_kernel_harness.cpp): the candidate geom pairs in
// the order the serial mj_collision emits their contacts, each with what mj_collideGeoms
// derives from the model alone. Read by the cooperative constraint kernel (its pair program)
// and by the generic collision() (engine_device.h), which then tests only the bounding
// spheres per instance.
#ifndef MJHIP_PAIR_PROGRAM_H_
#define MJHIP_PAIR_PROGRAM_H_

#include <algorithm>
#include <utility>
#include <vector>

#include "engine_device.h"

// one candidate geom pair: its geoms (body order) and its predefined-pair index, or -1
struct ProgItem {
  int g1, g2, ipair;
};

// The static geom-pair program of mj_collision (engine_collision_driver.c:265-497) for the
// cooperative constraint kernel and collision(): candidate body pairs in signature order (mjhip_contact.h),
// their geoms all-to-all, minus the pairs no run can collide (no collision function, geom
// bitmask); a body pair the midphase handles (a body with more than one geom) has its geom
// pairs stably sorted by contactcompare's key (:227-257), the type-ordered geom ids. Every
// contact of a pair carries that key, so this is the order the serial collision() leaves
// its contacts in, and the cooperative kernel concatenates the pairs' contacts in it.
// Predefined pairs (ipair = the pair's index, else -1) merge in as the device collision() does:
// ahead of the first body pair whose signature is not below theirs, the rest at the end, and
// a candidate's geom pair that is a predefined pair is left to it.
inline std::vector<ProgItem> collision_pairs(const mjhipModel* m) {
  std::vector<ProgItem> out;
  if (!mjhip_contactsEnabled(m)) return out;
  int pairadr = 0;
  auto predefined = [&](int k) {
    const int g1 = m->pair_geom1[k], g2 = m->pair_geom2[k];
    const bool flip = m->geom_type[g1] > m->geom_type[g2];
    if (mjhip_pairMaxContacts(m, m->geom_type[flip ? g2 : g1], m->geom_type[flip ? g1 : g2])) {
      out.push_back(ProgItem{g1, g2, k});
    }
  };
  const bool midphase = !(m->opt.disableflags & mjhipDSBL_MIDPHASE);
  auto key = [&](const ProgItem& p) {
    return m->geom_type[p.g1] > m->geom_type[p.g2] ? std::make_pair(p.g2, p.g1)
                                                   : std::make_pair(p.g1, p.g2);
  };
  for (int b1 = 0; b1 < m->nbody; b1++) {
    for (int b2 = b1 + 1; b2 < m->nbody; b2++) {
      for (; pairadr < m->npair && m->pair_signature[pairadr] <= (b1 << 16) + b2; pairadr++) {
        predefined(pairadr);
      }
      if (!mjhip_bodyPairCandidate(m, b1, b2)) continue;
      const int n1 = m->body_geomnum[b1], n2 = m->body_geomnum[b2];
      std::vector<ProgItem> list;
      for (int i = 0; i < n1; i++) {
        for (int j = 0; j < n2; j++) {
          const int g1 = m->body_geomadr[b1] + i, g2 = m->body_geomadr[b2] + j;
          if (m->npair && mjhip_isPredefinedPair(m, g1, g2)) continue;
          const std::pair<int, int> k = key(ProgItem{g1, g2, -1});
          if (!mjhip_pairMaxContacts(m, m->geom_type[k.first], m->geom_type[k.second])) continue;
          if (mjhip_filterBitmask(m->geom_contype[g1], m->geom_conaffinity[g1],
                                  m->geom_contype[g2], m->geom_conaffinity[g2])) {
            continue;
          }
          list.push_back(ProgItem{g1, g2, -1});
        }
      }
      if (midphase && !(n1 == 1 && n2 == 1)) {
        std::stable_sort(list.begin(), list.end(),
                         [&](const ProgItem& a, const ProgItem& b) { return key(a) < key(b); });
      }
      out.insert(out.end(), list.begin(), list.end());
    }
  }
  for (; pairadr < m->npair; pairadr++) predefined(pairadr);
  return out;
}

// the cooperative kernel's program for collision_pairs' pairs: what mj_collideGeoms derives
// from the model alone, type-ordered as narrowGeoms does (engine_collision_driver.c:1440-1497)
inline std::vector<CoopPair> coop_program(const mjhipModel* m,
                                          const std::vector<ProgItem>& pairs) {
  std::vector<CoopPair> out;
  const bool ovr = (m->opt.enableflags & mjhipENBL_OVERRIDE) != 0;
  for (const ProgItem& pr : pairs) {
    CoopPair P{};
    P.g1 = pr.g1;
    P.g2 = pr.g2;
    if (m->geom_type[P.g1] > m->geom_type[P.g2]) std::swap(P.g1, P.g2);
    P.t1 = m->geom_type[P.g1];
    P.t2 = m->geom_type[P.g2];
    P.kmax = mjhip_pairMaxContacts(m, P.t1, P.t2);
    P.b1 = m->geom_bodyid[P.g1];
    P.b2 = m->geom_bodyid[P.g2];
    P.rt1 = m->body_rootid[P.b1];
    P.rt2 = m->body_rootid[P.b2];
    const double mg1 = m->geom_margin[P.g1], mg2 = m->geom_margin[P.g2];
    P.margin = ovr ? m->opt.o_margin : pr.ipair >= 0 ? m->pair_margin[pr.ipair] : (mg1 > mg2 ? mg1 : mg2);
    const double rb1 = m->geom_rbound[P.g1], rb2 = m->geom_rbound[P.g2];
    if (rb1 > 0 && rb2 > 0) {
      P.filt = 0;
      P.bound = rb1 + rb2 + P.margin;
    } else if (P.t1 == mjhipGEOM_PLANE && rb2 > 0) {
      P.filt = 1;
      P.bound = P.margin + rb2;
    } else if (P.t2 == mjhipGEOM_PLANE && rb1 > 0) {
      P.filt = 2;
      P.bound = P.margin + rb1;
    } else {
      P.filt = 3;
    }
    out.push_back(P);
  }
  return out;
}

// each program entry's contact parameters (mjh::pairParam: a predefined pair's own, else
// mj_contactParam's mix): model constants, formed once by the same function
inline std::vector<mjh::ContactParam> program_params(const mjhipModel* m,
                                                     const std::vector<CoopPair>& prog,
                                                     const std::vector<ProgItem>& items) {
  std::vector<mjh::ContactParam> cps(prog.size());
  for (size_t i = 0; i < prog.size(); i++) {
    mjh::pairParam(*m, prog[i].g1, prog[i].g2, items[i].ipair, cps[i]);
  }
  return cps;
}

#endif  // MJHIP_PAIR_PROGRAM_H_
