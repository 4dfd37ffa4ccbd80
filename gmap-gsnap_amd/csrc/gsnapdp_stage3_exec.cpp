// gsnapdp_stage3_exec.cpp -- the stage-3 passes' batch executor on the GPU
// (gsnapdp_stage3.h).  A slot is one packed round: page-locked input and output
// staging, device buffers of the same layout and an event.  submit() is one H2D
// copy, the four families' device pipelines (gsnapdp_run_device -> k_plan /
// k_fill / k_rows, gsnapdp_ggap_run_device -> k_ggap_plan / k_gband / k_ggap,
// gsnapdp_cgap_run_device, gsnapdp_micro_run_device) back to back on the
// context stream, one D2H copy of every result and op stream, and an event
// record: one synchronisation per round instead of one per family, and nothing
// blocks the host until wait().  The families share the context's scratch, so
// every slot of every executor uses the one context stream (FIFO), which is
// also what makes concurrent passes on one context safe.  The launches
// themselves (≈20 runtime calls, ≈140 us of host time per round) run on the
// executor's own launcher thread, in submission order, so that the pass's
// threads resume the other cohort meanwhile; wait() first waits for the
// round's launches, then for its event.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gsnapdp_ctx.h"
#include "gsnapdp_stage3.h"

namespace gsnapdp {
namespace {

// GSNAPDP_S3_RECORD=DIR: every round's layout and output staging, in order
// (DIR/round_NNNNNN.bin), so that the pass's host work can be replayed and
// profiled on a machine without a GPU (tests/dropin/stage3_exec_replay.cpp)
const char* record_dir() {
  static const char* d = getenv("GSNAPDP_S3_RECORD");
  return d;
}
std::atomic<int> g_round{0};

struct Slot {
  char* h_in = nullptr;
  char* h_out = nullptr;
  char* d_in = nullptr;
  char* d_out = nullptr;
  size_t in_cap = 0, out_cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;
  bool launched = false;  // the launcher thread has issued the round (guarded by the executor's mutex)
  int rc = 0;             // and its result, with the launcher's error message
  std::string err;
  S3Layout L;  // the round in flight (for recording)
};

class GpuExec final : public S3Exec {
 public:
  explicit GpuExec(gsnapdp_ctx* ctx) : ctx_(ctx) {}
  ~GpuExec() override {
    if (th_.joinable()) {
      {
        std::lock_guard<std::mutex> l(m_);
        stop_ = true;
      }
      cv_.notify_all();
      th_.join();
    }
    for (Slot& s : slot_) {
      if (s.ev) (void)hipEventSynchronize(s.ev), (void)hipEventDestroy(s.ev);
      if (s.h_in) (void)hipHostFree(s.h_in);
      if (s.h_out) (void)hipHostFree(s.h_out);
      (void)hipFree(s.d_in);
      (void)hipFree(s.d_out);
    }
  }
  char* in_buf(int k, size_t bytes) override {
    Slot& s = slot_[k];
    if (bytes > s.in_cap) {
      const size_t cap = grow(bytes);
      if (s.h_in) (void)hipHostFree(s.h_in);
      (void)hipFree(s.d_in);
      s.h_in = s.d_in = nullptr;
      s.in_cap = 0;
      if (hipHostMalloc(&s.h_in, cap) != hipSuccess || hipMalloc(&s.d_in, cap) != hipSuccess) {
        gsnapdp__set_err("stage-3 executor: input staging allocation failed");
        return nullptr;
      }
      s.in_cap = cap;
    }
    return s.h_in;
  }
  char* out_buf(int k, size_t bytes) override {
    Slot& s = slot_[k];
    if (bytes > s.out_cap) {
      const size_t cap = grow(bytes);
      if (s.h_out) (void)hipHostFree(s.h_out);
      (void)hipFree(s.d_out);
      s.h_out = s.d_out = nullptr;
      s.out_cap = 0;
      if (hipHostMalloc(&s.h_out, cap) != hipSuccess || hipMalloc(&s.d_out, cap) != hipSuccess) {
        gsnapdp__set_err("stage-3 executor: output staging allocation failed");
        return nullptr;
      }
      s.out_cap = cap;
    }
    return s.h_out;
  }
  int submit(int k, const S3Layout& L) override {
    Slot& s = slot_[k];
    if (L.in_bytes > s.in_cap || L.out_bytes > s.out_cap) {
      gsnapdp__set_err("stage-3 executor: layout larger than its staging");
      return -1;
    }
    if (!th_.joinable()) th_ = std::thread([this] { launcher(); });
    {
      std::lock_guard<std::mutex> l(m_);
      s.L = L;
      s.pending = true;
      s.launched = false;
      q_.push_back(k);
    }
    cv_.notify_all();
    return 0;
  }
  int wait(int k) override {
    Slot& s = slot_[k];
    if (!s.pending) return 0;
    s.pending = false;
    {
      std::unique_lock<std::mutex> l(m_);
      cv_.wait(l, [&] { return s.launched; });
    }
    if (s.rc) {
      gsnapdp__set_err(s.err);
      return -1;
    }
    HIPCHK(hipEventSynchronize(s.ev));
    if (record_dir()) {
      char path[4096];
      snprintf(path, sizeof(path), "%s/round_%06d.bin", record_dir(), g_round.fetch_add(1));
      if (FILE* f = fopen(path, "wb")) {
        fwrite(&s.L, sizeof(s.L), 1, f);
        fwrite(s.h_out, 1, s.L.out_bytes, f);
        fclose(f);
      }
    }
    return 0;
  }

 private:
  void launcher() {
    for (;;) {
      int k;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        k = q_.front();
        q_.pop_front();
      }
      Slot& s = slot_[k];
      const int rc = launch(s);
      {
        std::lock_guard<std::mutex> l(m_);
        s.rc = rc;
        s.err = rc ? gsnapdp_last_error() : "";
        s.launched = true;
      }
      cv_.notify_all();
    }
  }
  // one H2D copy, every family's device pipeline, one D2H copy and the event
  int launch(Slot& s) {
    const S3Layout& L = s.L;
    HIPCHK(hipSetDevice(ctx_->device));
    if (!s.ev) HIPCHK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
    hipStream_t st = ctx_->stream;
    HIPCHK(hipMemcpyAsync(s.d_in, s.h_in, L.in_bytes, hipMemcpyHostToDevice, st));
    const char* dq = s.d_in + L.q;
    const char* du = s.d_in + L.qu;
    auto off = [&](int f) { return (const int64_t*)(s.d_in + L.off[f]); };
    if (L.n[S3F_GAP] &&
        gsnapdp_run_device(ctx_, (const gsnapdp_window*)(s.d_in + L.w[S3F_GAP]), L.n[S3F_GAP], dq, du,
                           (gsnapdp_result*)(s.d_out + L.r[S3F_GAP]), (uint32_t*)(s.d_out + L.ops[S3F_GAP]),
                           off(S3F_GAP), st))
      return -1;
    if (L.n[S3F_GGAP] &&
        gsnapdp_ggap_run_device(ctx_, (const gsnapdp_ggap_window*)(s.d_in + L.w[S3F_GGAP]), L.n[S3F_GGAP], dq,
                                du, (gsnapdp_ggap_result*)(s.d_out + L.r[S3F_GGAP]),
                                (gsnapdp_ggap_trace*)(s.d_out + L.t), (uint32_t*)(s.d_out + L.ops[S3F_GGAP]),
                                off(S3F_GGAP), st))
      return -1;
    if (L.n[S3F_CGAP] &&
        gsnapdp_cgap_run_device(ctx_, (const gsnapdp_cgap_window*)(s.d_in + L.w[S3F_CGAP]), L.n[S3F_CGAP], dq,
                                du, (gsnapdp_cgap_result*)(s.d_out + L.r[S3F_CGAP]),
                                (uint32_t*)(s.d_out + L.ops[S3F_CGAP]), off(S3F_CGAP), st))
      return -1;
    if (L.n[S3F_MICRO] &&
        gsnapdp_micro_run_device(ctx_, (const gsnapdp_micro_window*)(s.d_in + L.w[S3F_MICRO]), L.n[S3F_MICRO],
                                 dq, du, (gsnapdp_micro_result*)(s.d_out + L.r[S3F_MICRO]), st))
      return -1;
    HIPCHK(hipMemcpyAsync(s.h_out, s.d_out, L.out_bytes, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(s.ev, st));
    return 0;
  }
  static size_t grow(size_t bytes) {  // room for the next few rounds without reallocating
    size_t cap = (size_t)1 << 20;
    while (cap < bytes + bytes / 4) cap <<= 1;
    return cap;
  }
  gsnapdp_ctx* ctx_;
  Slot slot_[2];
  std::thread th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<int> q_;
  bool stop_ = false;
};

}  // namespace

S3Exec* s3_exec_acquire(gsnapdp_ctx* ctx) {
  std::lock_guard<std::mutex> lock(ctx->s3_mu);
  if (!ctx->s3_pool.empty()) {
    S3Exec* e = (S3Exec*)ctx->s3_pool.back();
    ctx->s3_pool.pop_back();
    return e;
  }
  return new GpuExec(ctx);
}

gsnapdp_s3_stage2 s3_stage2(gsnapdp_ctx* ctx) {
  std::lock_guard<std::mutex> lock(ctx->s3_mu);
  return ctx->s3_stage2;
}
void s3_set_stage2(gsnapdp_ctx* ctx, const gsnapdp_s3_stage2& s2) {
  std::lock_guard<std::mutex> lock(ctx->s3_mu);
  ctx->s3_stage2 = s2;
}

void s3_exec_release(gsnapdp_ctx* ctx, S3Exec* e) {
  if (!e) return;
  std::lock_guard<std::mutex> lock(ctx->s3_mu);
  ctx->s3_pool.push_back((void*)e);
}

}  // namespace gsnapdp

void gsnapdp__s3_pool_free(gsnapdp_ctx* ctx) {
  std::lock_guard<std::mutex> lock(ctx->s3_mu);
  for (void* p : ctx->s3_pool) delete (gsnapdp::S3Exec*)p;
  ctx->s3_pool.clear();
}
