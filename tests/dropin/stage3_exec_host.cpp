// stage3_exec_host.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never on a GPU box).
//
// The stage-3 passes' batch executor (gmap-gsnap_amd/csrc/gsnapdp_stage3.h)
// for the CPU build of the pass (oracle/Makefile `stage3_cpu`): the same
// packed round layout the GPU executor stages through page-locked memory,
// served synchronously by the host entry points, which the oracle's
// restatement provides there (tests/dropin/gsnapdp_oracle_abi.c).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <vector>

#include "../../gmap-gsnap_amd/csrc/gsnapdp_stage3.h"

// seconds spent serving batches (the oracle's DP), for timing the pass's own host work
double g_s3_exec_seconds = 0.0;

namespace gsnapdp {
namespace {

class HostExec final : public S3Exec {
 public:
  explicit HostExec(gsnapdp_ctx* ctx) : ctx_(ctx) {}
  char* in_buf(int k, size_t bytes) override {
    if (in_[k].size() < bytes) in_[k].resize(bytes);
    return in_[k].data();
  }
  char* out_buf(int k, size_t bytes) override {
    if (out_[k].size() < bytes) out_[k].resize(bytes);
    return out_[k].data();
  }
  int submit(int k, const S3Layout& L) override {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = serve(k, L);
    g_s3_exec_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
  }
  int wait(int) override { return 0; }

 private:
  // every family's windows in chunks on the pass's host threads (the oracle's
  // batch drivers are reentrant: one workspace per call)
  int serve(int k, const S3Layout& L) {
    char* in = in_[k].data();
    char* out = out_[k].data();
    const char* q = in + L.q;
    const char* qu = in + L.qu;
    auto off = [&](int f) { return (const int64_t*)(in + L.off[f]); };
    std::vector<int> jf, jlo, jhi;
    for (int f = 0; f < S3F_N; f++)
      for (int lo = 0; lo < L.n[f]; lo += kChunk) {
        jf.push_back(f);
        jlo.push_back(lo);
        jhi.push_back(std::min(L.n[f], lo + kChunk));
      }
    std::atomic<int> bad(0);
    s3_parallel_for((int)jf.size(), 1, [&](int j) {
      const int f = jf[(size_t)j], lo = jlo[(size_t)j], n = jhi[(size_t)j] - lo;
      int rc = 0;
      if (f == S3F_GAP)
        rc = gsnapdp_run_host(ctx_, (const gsnapdp_window*)(in + L.w[f]) + lo, n, q, qu, L.qbytes,
                              (gsnapdp_result*)(out + L.r[f]) + lo, (uint32_t*)(out + L.ops[f]), off(f) + lo);
      else if (f == S3F_GGAP)
        rc = gsnapdp_ggap_run_host(ctx_, (const gsnapdp_ggap_window*)(in + L.w[f]) + lo, n, q, qu, L.qbytes,
                                   (gsnapdp_ggap_result*)(out + L.r[f]) + lo, (gsnapdp_ggap_trace*)(out + L.t) + lo,
                                   (uint32_t*)(out + L.ops[f]), off(f) + lo);
      else if (f == S3F_CGAP)
        rc = gsnapdp_cgap_run_host(ctx_, (const gsnapdp_cgap_window*)(in + L.w[f]) + lo, n, q, qu, L.qbytes,
                                   (gsnapdp_cgap_result*)(out + L.r[f]) + lo, (uint32_t*)(out + L.ops[f]),
                                   off(f) + lo);
      else
        rc = gsnapdp_micro_run_host(ctx_, (const gsnapdp_micro_window*)(in + L.w[f]) + lo, n, q, qu, L.qbytes,
                                    (gsnapdp_micro_result*)(out + L.r[f]) + lo);
      if (rc) bad.store(1);
    });
    return bad.load() ? -1 : 0;
  }
  static constexpr int kChunk = 64;
  gsnapdp_ctx* ctx_;
  std::vector<char> in_[2], out_[2];
};

}  // namespace

S3Exec* s3_exec_acquire(gsnapdp_ctx* ctx) { return new HostExec(ctx); }
void s3_exec_release(gsnapdp_ctx*, S3Exec* e) { delete e; }

// the stage-2 callback (one per process in the test builds)
static std::mutex g_s2_mu;
static gsnapdp_s3_stage2 g_s2 = {nullptr, nullptr};
gsnapdp_s3_stage2 s3_stage2(gsnapdp_ctx*) {
  std::lock_guard<std::mutex> l(g_s2_mu);
  return g_s2;
}
void s3_set_stage2(gsnapdp_ctx*, const gsnapdp_s3_stage2& s2) {
  std::lock_guard<std::mutex> l(g_s2_mu);
  g_s2 = s2;
}

}  // namespace gsnapdp
