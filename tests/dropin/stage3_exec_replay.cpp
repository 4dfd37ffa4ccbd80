// stage3_exec_replay.cpp -- TEST / PROFILING INFRASTRUCTURE ONLY (never shipped).
//
// The stage-3 passes' batch executor (gmap-gsnap_amd/csrc/gsnapdp_stage3.h)
// replaying the rounds a GPU run recorded (GSNAPDP_S3_RECORD=DIR,
// gsnapdp_stage3_exec.cpp): each submit() takes the next recorded round, checks
// that the pass packed the same batch, and copies the GPU's outputs into the
// slot.  The pass's host work (peels, traversals, the product's op-stream
// expansion) then runs exactly as on the GPU box, on a machine without one
// (tools/s3_host_profile.sh).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <mutex>
#include <vector>

#include "../../gmap-gsnap_amd/csrc/gsnapdp_stage3.h"

namespace gsnapdp {
namespace {

int g_next = 0;

class ReplayExec final : public S3Exec {
 public:
  char* in_buf(int k, size_t bytes) override {
    if (in_[k].size() < bytes) in_[k].resize(bytes);
    return in_[k].data();
  }
  char* out_buf(int k, size_t bytes) override {
    if (out_[k].size() < bytes) out_[k].resize(bytes);
    return out_[k].data();
  }
  int submit(int k, const S3Layout& L) override {
    const char* dir = getenv("GSNAPDP_S3_REPLAY");
    char path[4096];
    snprintf(path, sizeof(path), "%s/round_%06d.bin", dir ? dir : ".", g_next++);
    FILE* f = fopen(path, "rb");
    if (!f) {
      fprintf(stderr, "replay executor: no recorded %s\n", path);
      return -1;
    }
    S3Layout R;
    bool ok = fread(&R, sizeof(R), 1, f) == 1;
    for (int i = 0; i < S3F_N; i++) ok = ok && R.n[i] == L.n[i] && R.ops[i] == L.ops[i];
    ok = ok && R.out_bytes == L.out_bytes && out_[k].size() >= L.out_bytes;
    ok = ok && fread(out_[k].data(), 1, L.out_bytes, f) == L.out_bytes;
    fclose(f);
    if (!ok) fprintf(stderr, "replay executor: %s does not match the packed round\n", path);
    return ok ? 0 : -1;
  }
  int wait(int) override { return 0; }

 private:
  std::vector<char> in_[2], out_[2];
};

}  // namespace

S3Exec* s3_exec_acquire(gsnapdp_ctx*) {
  g_next = 0;  // every pass replays the recorded pass from its first round
  return new ReplayExec();
}
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
