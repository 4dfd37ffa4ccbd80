// stage3_cpu_driver.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never on a GPU box).
//
// Runs gsnapdp_stage3_pass (gmap-gsnap_amd/csrc/gsnapdp_stage3.cpp) on the CPU,
// its gap families served by the oracle's restatement
// (tests/dropin/gsnapdp_oracle_abi.c), under AddressSanitizer + UBSan
// (oracle/Makefile `stage3_cpu`).  tests/test_stage3_cpu.py feeds it the
// build_pairs_introns calls gmap_trace recorded and compares the lists.
//
//   stage3_cpu DIR    reads DIR/{calls,pairs_in,query,query_uc}.bin, DIR/genome.u32 and, when
//                     present, DIR/intervals.bin (gsnapdp_iit_interval: a splicing IIT) and
//                     DIR/stage2_{calls,pairs}.bin (traverse_dual_break's recorded stage-2 lists);
//                     writes DIR/{pass_calls,pass_pairs,pass_stats}.bin, and with
//                     --introns DIR/pass_scores.bin (score_introns on the returned lists);
//   stage3_cpu DIR --compute MINLEN   passes 2A-6 (gsnapdp_stage3_compute) over the queries in
//                     calls.bin: DIR/{pass_calls,pass_pairs,compute_stats}.bin
//   stage3_cpu DIR --path-compute MINLEN MAXINTRONLEN [GSNAP]   path_compute from pass 2A to its return
//                     value (gsnapdp_stage3_path_compute): the same files and DIR/pass_probs.bin
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/gsnapdp.h"

extern "C" {
void* s2dbl_new(const void* calls, int ncalls, const gsnapdp_s3_pair* pairs, int npairs);
int s2dbl_compute_one(void* u, const gsnapdp_s3_call* call, int querydp5, int querydp3, int genomedp5,
                      int genomedp3, uint32_t mappingstart, uint32_t mappingend, gsnapdp_s3_pair* out, int cap);
}

static std::string g_err;
extern double g_s3_exec_seconds;  // stage3_exec_host.cpp
void gsnapdp__set_err(const std::string& s) { g_err = s; }

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
template <class T>
static void spit(const std::string& path, const T* p, size_t n) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f || (n && fwrite(p, sizeof(T), n, f) != n)) exit(3);
  fclose(f);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string d = argv[1];
  const bool introns = argc > 2 && std::string(argv[2]) == "--introns";
  // --compute MINLEN: gsnapdp_stage3_compute with min_intronlength MINLEN
  const int compute = argc > 3 && std::string(argv[2]) == "--compute" ? atoi(argv[3]) : -1;
  // --path-compute MINLEN MAXINTRONLEN: gsnapdp_stage3_path_compute
  const bool path_compute = argc > 4 && std::string(argv[2]) == "--path-compute";
  std::vector<gsnapdp_s3_call> calls = slurp<gsnapdp_s3_call>(d + "/calls.bin");
  std::vector<gsnapdp_s3_pair> in = slurp<gsnapdp_s3_pair>(d + "/pairs_in.bin");
  std::vector<char> q = slurp<char>(d + "/query.bin"), qu = slurp<char>(d + "/query_uc.bin");
  std::vector<uint32_t> blocks = slurp<uint32_t>(d + "/genome.u32");
  std::vector<double> tables = slurp<double>(getenv("GSNAPDP_MAXENT_TABLES"));
  gsnapdp_ctx* ctx = gsnapdp_create(0, blocks.data(), blocks.size(), 0);
  if (!ctx || gsnapdp_load_maxent_tables(ctx, tables.data(), tables.size())) return 4;
  int64_t cap = 0;
  for (const gsnapdp_s3_call& c : calls) cap += 2 * ((int64_t)c.querylength + c.npairs) + 64;
  std::vector<gsnapdp_s3_pair> out((size_t)cap);
  gsnapdp_s3_stats st;
  gsnapdp_iit* iit = nullptr;
  if (FILE* f = fopen((d + "/intervals.bin").c_str(), "rb")) {
    fclose(f);
    std::vector<gsnapdp_iit_interval> iv = slurp<gsnapdp_iit_interval>(d + "/intervals.bin");
    if (!(iit = gsnapdp_iit_from_intervals(iv.data(), (int)iv.size()))) return 4;
  }
  void* s2 = nullptr;  // traverse_dual_break's stage-2 lists, from the recording (stage2_double.c)
  if (FILE* f = fopen((d + "/stage2_calls.bin").c_str(), "rb")) {
    fclose(f);
    std::vector<char> sc = slurp<char>(d + "/stage2_calls.bin");
    std::vector<gsnapdp_s3_pair> sp = slurp<gsnapdp_s3_pair>(d + "/stage2_pairs.bin");
    s2 = s2dbl_new(sc.data(), (int)(sc.size() / 48), sp.data(), (int)sp.size());
    gsnapdp_s3_stage2 cb = {s2, s2dbl_compute_one};
    gsnapdp_stage3_set_stage2(ctx, &cb);
  }
  if (path_compute) {  // pass 2A to path_compute's return value: calls.bin holds the queries
    gsnapdp_s3_compute_stats cs;
    gsnapdp_s3_path_opts o = {};
    o.min_intronlength = atoi(argv[3]);
    o.maxintronlen_bound = atoi(argv[4]);
    o.gsnap = argc > 5 ? atoi(argv[5]) : 0;  // 1: stage3.c as GSNAP builds it
    std::vector<gsnapdp_s3_pair> big((size_t)cap * 2 + 1024);
    std::vector<double> probs(big.size() * 2);
    if (gsnapdp_stage3_path_compute(ctx, calls.data(), (int)calls.size(), in.data(), (int64_t)in.size(), q.data(),
                                    qu.data(), std::min(q.size(), qu.size()), iit, &o, big.data(),
                                    (int64_t)big.size(), probs.data(), &cs)) {
      fprintf(stderr, "gsnapdp_stage3_path_compute: %s\n", g_err.c_str());
      return 5;
    }
    fprintf(stderr, "path_compute %.4f s (host steps %.4f, passes %.4f), %d passes, %d rounds, %d sites, %d failed\n",
            cs.seconds[2], cs.seconds[0], cs.seconds[1], cs.passes, cs.rounds, cs.sites, cs.failed);
    int64_t nout = 0;
    for (const gsnapdp_s3_call& c : calls) nout += c.nout;
    spit(d + "/pass_calls.bin", calls.data(), calls.size());
    spit(d + "/pass_pairs.bin", big.data(), (size_t)nout);
    spit(d + "/pass_probs.bin", probs.data(), (size_t)nout * 2);
    spit(d + "/compute_stats.bin", &cs, 1);
    gsnapdp_destroy(ctx);
    return 0;
  }
  if (compute >= 0) {  // passes 2A-6 (gsnapdp_stage3_compute): calls.bin holds the queries
    gsnapdp_s3_compute_stats cs;
    std::vector<gsnapdp_s3_pair> big((size_t)cap * 2 + 1024);
    if (gsnapdp_stage3_compute(ctx, calls.data(), (int)calls.size(), in.data(), (int64_t)in.size(), q.data(),
                               qu.data(), std::min(q.size(), qu.size()), iit, compute, big.data(),
                               (int64_t)big.size(), &cs)) {
      fprintf(stderr, "gsnapdp_stage3_compute: %s\n", g_err.c_str());
      return 5;
    }
    fprintf(stderr, "compute %.4f s (host steps %.4f, passes %.4f), %d passes, %d rounds, %d failed\n",
            cs.seconds[2], cs.seconds[0], cs.seconds[1], cs.passes, cs.rounds, cs.failed);
    int64_t nout = 0;
    for (const gsnapdp_s3_call& c : calls) nout += c.nout;
    spit(d + "/pass_calls.bin", calls.data(), calls.size());
    spit(d + "/pass_pairs.bin", big.data(), (size_t)nout);
    spit(d + "/compute_stats.bin", &cs, 1);
    gsnapdp_destroy(ctx);
    return 0;
  }
  // GSNAPDP_S3_REPS=N: N passes over the same calls (warm host timing: the later
  // passes reuse the pass's path store), each one's profile printed
  const int reps = getenv("GSNAPDP_S3_REPS") ? std::max(1, atoi(getenv("GSNAPDP_S3_REPS"))) : 1;
  for (int r = 0; r < reps; r++) {
    std::vector<gsnapdp_s3_call> cc = calls;
    g_s3_exec_seconds = 0;
    if (gsnapdp_stage3_pass(ctx, cc.data(), (int)cc.size(), in.data(), (int64_t)in.size(), q.data(), qu.data(),
                            std::min(q.size(), qu.size()), iit, out.data(), cap, &st)) {
      fprintf(stderr, "gsnapdp_stage3_pass: %s\n", g_err.c_str());
      return 5;
    }
    if (r == reps - 1) calls = cc;
    else
      fprintf(stderr, "rep %d: pass %.4f s, oracle %.4f s, host %.4f s\n", r, st.seconds[2], g_s3_exec_seconds,
              st.seconds[2] - g_s3_exec_seconds);
  }
  if (introns) {
    std::vector<gsnapdp_intron_scores> sc(calls.size());
    if (gsnapdp_stage3_score_introns(ctx, calls.data(), (int)calls.size(), out.data(), iit, sc.data())) {
      fprintf(stderr, "gsnapdp_stage3_score_introns: %s\n", g_err.c_str());
      return 6;
    }
    spit(d + "/pass_scores.bin", sc.data(), sc.size());
  }
  gsnapdp_iit_free(iit);
  fprintf(stderr, "pass %.4f s (host %.4f, waits %.4f), batches served by the oracle %.4f s, %d rounds\n",
          st.seconds[2], st.seconds[0], st.seconds[1], g_s3_exec_seconds, st.rounds);
  int64_t nout = 0;
  for (const gsnapdp_s3_call& c : calls) nout += c.nout;
  spit(d + "/pass_calls.bin", calls.data(), calls.size());
  spit(d + "/pass_pairs.bin", out.data(), (size_t)nout);
  spit(d + "/pass_stats.bin", &st, 1);
  gsnapdp_destroy(ctx);
  return 0;
}
