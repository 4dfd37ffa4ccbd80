// stage3_exec_host.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never on a GPU box).
//
// The stage-3 passes' batch executor (gmap-gsnap_amd/csrc/gsnapdp_stage3.h)
// for the CPU build of the pass (oracle/Makefile `stage3_cpu`): the same
// packed round layout the GPU executor stages through page-locked memory,
// served synchronously by the host entry points, which the oracle's
// restatement provides there (tests/dropin/gsnapdp_oracle_abi.c).
#include <chrono>
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
  int serve(int k, const S3Layout& L) {
    char* in = in_[k].data();
    char* out = out_[k].data();
    const char* q = in + L.q;
    const char* qu = in + L.qu;
    auto off = [&](int f) { return (const int64_t*)(in + L.off[f]); };
    if (L.n[S3F_GAP] && gsnapdp_run_host(ctx_, (const gsnapdp_window*)(in + L.w[S3F_GAP]), L.n[S3F_GAP], q, qu,
                                         L.qbytes, (gsnapdp_result*)(out + L.r[S3F_GAP]),
                                         (uint32_t*)(out + L.ops[S3F_GAP]), off(S3F_GAP)))
      return -1;
    if (L.n[S3F_GGAP] &&
        gsnapdp_ggap_run_host(ctx_, (const gsnapdp_ggap_window*)(in + L.w[S3F_GGAP]), L.n[S3F_GGAP], q, qu,
                              L.qbytes, (gsnapdp_ggap_result*)(out + L.r[S3F_GGAP]),
                              (gsnapdp_ggap_trace*)(out + L.t), (uint32_t*)(out + L.ops[S3F_GGAP]), off(S3F_GGAP)))
      return -1;
    if (L.n[S3F_CGAP] &&
        gsnapdp_cgap_run_host(ctx_, (const gsnapdp_cgap_window*)(in + L.w[S3F_CGAP]), L.n[S3F_CGAP], q, qu,
                              L.qbytes, (gsnapdp_cgap_result*)(out + L.r[S3F_CGAP]),
                              (uint32_t*)(out + L.ops[S3F_CGAP]), off(S3F_CGAP)))
      return -1;
    if (L.n[S3F_MICRO] &&
        gsnapdp_micro_run_host(ctx_, (const gsnapdp_micro_window*)(in + L.w[S3F_MICRO]), L.n[S3F_MICRO], q, qu,
                               L.qbytes, (gsnapdp_micro_result*)(out + L.r[S3F_MICRO])))
      return -1;
    return 0;
  }
  gsnapdp_ctx* ctx_;
  std::vector<char> in_[2], out_[2];
};

}  // namespace

S3Exec* s3_exec_acquire(gsnapdp_ctx* ctx) { return new HostExec(ctx); }
void s3_exec_release(gsnapdp_ctx*, S3Exec* e) { delete e; }

}  // namespace gsnapdp
