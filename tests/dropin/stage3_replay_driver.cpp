// stage3_replay_driver.cpp -- PROFILING INFRASTRUCTURE ONLY (never shipped, never on a GPU box).
//
// Runs gsnapdp_stage3_pass with the product's host code -- the pass
// (gsnapdp_stage3.cpp) and the op-stream expanders (gsnapdp_host.cpp) -- over
// the rounds a GPU run recorded (tools/s3_record.py; the replay executor,
// tests/dropin/stage3_exec_replay.cpp), so that the pass's host work can be
// timed and profiled here.  oracle/Makefile `stage3_host_replay`.
//
//   stage3_host_replay DIR [REPS]   DIR holds the recorded pass: calls.bin pairs_in.bin
//                                   query.bin query_uc.bin genome.u32 round_*.bin;
//                                   checks every rep's lists against DIR/pairs_out.bin
//                                   (with DIR/gaps.bin + gap_off.bin: the runs-mode pass,
//                                   checked against DIR/runs_out.bin + new_out.bin)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "../../gmap-gsnap_amd/csrc/gsnapdp_internal.h"
#include "../../include/gsnapdp.h"

namespace gsnapdp {
void build_profile_table(int mode, uint32_t prof[PROF_WORDS]);  // pairdistance_init's tables too
}  // namespace gsnapdp

struct gsnapdp_ctx {
  const uint32_t* blocks;
  size_t nwords;
  uint32_t prof[gsnapdp::PROF_WORDS];
};
extern "C" const uint32_t* gsnapdp__host_blocks(gsnapdp_ctx* c) { return c->blocks; }
extern "C" size_t gsnapdp__host_nwords(gsnapdp_ctx* c) { return c->nwords; }
extern "C" const uint32_t* gsnapdp__host_prof(gsnapdp_ctx* c) { return c->prof; }
static std::string g_err;
void gsnapdp__set_err(const std::string& s) { g_err = s; }
extern "C" const char* gsnapdp_last_error(void) { return g_err.c_str(); }
extern "C" int gsnapdp_score_introns_host(gsnapdp_ctx*, const gsnapdp_intron_path*, int, const gsnapdp_intron*, int,
                                          gsnapdp_intron_scores*) {
  abort();  // not replayed
}

template <class T>
static std::vector<T> slurp(const std::string& path) {
  std::vector<T> v;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) {
    perror(path.c_str());
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  v.resize((size_t)n / sizeof(T) + 1);
  if (n && fread(v.data(), 1, (size_t)n, f) != (size_t)n) exit(2);
  fclose(f);
  v.resize((size_t)n / sizeof(T));
  return v;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string d = argv[1];
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  setenv("GSNAPDP_S3_REPLAY", d.c_str(), 1);
  std::vector<gsnapdp_s3_call> calls0 = slurp<gsnapdp_s3_call>(d + "/calls.bin");
  std::vector<gsnapdp_s3_pair> in = slurp<gsnapdp_s3_pair>(d + "/pairs_in.bin");
  std::vector<gsnapdp_s3_pair> want = slurp<gsnapdp_s3_pair>(d + "/pairs_out.bin");
  std::vector<char> q = slurp<char>(d + "/query.bin"), qu = slurp<char>(d + "/query_uc.bin");
  std::vector<uint32_t> blocks = slurp<uint32_t>(d + "/genome.u32");
  gsnapdp_ctx ctx;
  ctx.blocks = blocks.data();
  ctx.nwords = blocks.size();
  gsnapdp::build_profile_table(0, ctx.prof);
  // runs mode (gsnapdp_stage3_pass_runs) when the recording holds the caller's gap lists
  FILE* gf = fopen((d + "/gaps.bin").c_str(), "rb");
  if (gf) {
    fclose(gf);
    std::vector<int32_t> gaps = slurp<int32_t>(d + "/gaps.bin");
    std::vector<int64_t> gap_off = slurp<int64_t>(d + "/gap_off.bin");
    std::vector<gsnapdp_s3_run> want_runs = slurp<gsnapdp_s3_run>(d + "/runs_out.bin");
    std::vector<gsnapdp_s3_pair> want_new = slurp<gsnapdp_s3_pair>(d + "/new_out.bin");
    std::vector<gsnapdp_s3_run> runs(want_runs.size() + 1024);
    int64_t ncap = 0;
    for (const gsnapdp_s3_call& c : calls0) ncap += 2 * (int64_t)c.querylength + 256;
    std::unique_ptr<gsnapdp_s3_pair[]> news(new gsnapdp_s3_pair[(size_t)ncap]);  // (not zero-filled)
    for (int r = 0; r < reps; r++) {
      std::vector<gsnapdp_s3_call> calls = calls0;
      gsnapdp_s3_stats st;
      const auto t0 = std::chrono::steady_clock::now();
      if (gsnapdp_stage3_pass_runs(&ctx, calls.data(), (int)calls.size(), in.data(), (int64_t)in.size(), gaps.data(),
                                   gap_off.data(), q.data(), qu.data(), std::min(q.size(), qu.size()), nullptr,
                                   runs.data(), (int64_t)runs.size(), news.get(), ncap, &st)) {
        fprintf(stderr, "gsnapdp_stage3_pass_runs: %s\n", g_err.c_str());
        return 5;
      }
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      int64_t nout = 0;
      for (const gsnapdp_s3_call& c : calls) nout += c.nout;
      const bool same = (size_t)nout == want_runs.size() && (size_t)st.new_pairs == want_new.size() &&
                        !memcmp(runs.data(), want_runs.data(), want_runs.size() * sizeof(want_runs[0])) &&
                        !memcmp(news.get(), want_new.data(), want_new.size() * sizeof(want_new[0]));
      printf("rep %d: %zu paths in %.4f s = %.0f paths/s, %d rounds, runs %s\n", r, calls.size(), dt,
             calls.size() / dt, st.rounds, same ? "identical to the GPU run's" : "DIFFER");
      if (!same) return 6;
    }
    return 0;
  }
  int64_t cap = 0;
  for (const gsnapdp_s3_call& c : calls0) cap += 2 * ((int64_t)c.querylength + c.npairs) + 64;
  std::vector<gsnapdp_s3_pair> out((size_t)cap);
  for (int r = 0; r < reps; r++) {
    std::vector<gsnapdp_s3_call> calls = calls0;
    gsnapdp_s3_stats st;
    const auto t0 = std::chrono::steady_clock::now();
    if (gsnapdp_stage3_pass(&ctx, calls.data(), (int)calls.size(), in.data(), (int64_t)in.size(), q.data(),
                            qu.data(), std::min(q.size(), qu.size()), nullptr, out.data(), cap, &st)) {
      fprintf(stderr, "gsnapdp_stage3_pass: %s\n", g_err.c_str());
      return 5;
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    int64_t nout = 0;
    for (const gsnapdp_s3_call& c : calls) nout += c.nout;
    const bool same = (size_t)nout == want.size() && !memcmp(out.data(), want.data(), want.size() * sizeof(want[0]));
    printf("rep %d: %zu paths in %.4f s = %.0f paths/s, %d rounds, lists %s\n", r, calls.size(), dt,
           calls.size() / dt, st.rounds, same ? "identical to the GPU run's" : "DIFFER");
    if (!same) return 6;
  }
  return 0;
}
