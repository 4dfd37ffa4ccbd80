// gsnapdp_scan.cpp -- the MaxEnt half of GSNAP's splice-site scans
// (stage1hr.c:6300-7046, 8703-8976): the probability of every caller-supplied
// candidate site of many reads in one k_maxent launch (include/gsnapdp.h
// gsnapdp_scan_site_probs).  The candidate generation (Genome_donor_positions
// and the like) is defined in genome_hr.c, a missing blob of the reference, so
// it is not restated here (parity unpinned).  Host code.
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/gsnapdp.h"

void gsnapdp__set_err(const std::string& s);  // gsnapdp_kernels.hip

// GSNAP's splice-site scans, batched (include/gsnapdp.h gsnapdp_scan_site_probs):
// the known sites are 1.0 (stage1hr.c:6319-6334: `if (donori_knowni[i] >= 0)
// probi = 1.0`), the rest one k_maxent launch at segment_left + splice_pos.
extern "C" int gsnapdp_scan_site_probs(gsnapdp_ctx* ctx, const gsnapdp_scan_site* sites, int n, double* probs) {
  if (!ctx || n < 0 || (n > 0 && (!sites || !probs))) {
    gsnapdp__set_err("gsnapdp_scan_site_probs: bad arguments");
    return -1;
  }
  thread_local std::vector<uint8_t> model;
  thread_local std::vector<uint32_t> pos, chroff;
  thread_local std::vector<int> at;
  thread_local std::vector<double> p;
  model.clear(), pos.clear(), chroff.clear(), at.clear();
  for (int i = 0; i < n; i++) {
    const gsnapdp_scan_site& x = sites[i];
    if (x.knowni >= 0) {
      probs[i] = 1.0;
      continue;
    }
    if (x.model < GSNAPDP_DONOR || x.model > GSNAPDP_ANTIACCEPTOR) {
      gsnapdp__set_err("gsnapdp_scan_site_probs: site " + std::to_string(i) + " has no MaxEnt model");
      return -1;
    }
    model.push_back((uint8_t)x.model);
    pos.push_back(x.segment_left + (uint32_t)x.splice_pos);
    chroff.push_back(x.chroffset);
    at.push_back(i);
  }
  if (at.empty()) return 0;
  p.resize(at.size());
  if (gsnapdp_maxent_host(ctx, model.data(), pos.data(), chroff.data(), p.data(), (int)at.size())) return -1;
  for (size_t k = 0; k < at.size(); k++) probs[at[k]] = p[k];
  return 0;
}
