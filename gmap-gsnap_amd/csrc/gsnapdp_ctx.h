// gsnapdp_ctx.h -- the context behind gsnapdp_ctx* (host side), shared by
// gsnapdp_kernels.hip and gsnapdp_ggap.hip.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <vector>

#include "gsnapdp_internal.h"

void gsnapdp__set_err(const std::string& s);
struct gsnapdp_ctx;
// per-stage HIP events around a launch (gsnapdp_profile); stage < 16
void gsnapdp__mark(gsnapdp_ctx* ctx, hipStream_t st, int stage, int end);
// k_rows over the RW_NCLS row-lane class lists (gsnapdp_ggap.hip)
int gsnapdp__rows_launch(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_window* d_windows,
                         const int* lists, int* counts, int list_cap, const char* d_query,
                         const char* d_query_uc, gsnapdp_result* d_results, uint32_t* d_ops,
                         const int64_t* d_op_offsets, const gsnapdp_sj_window* sjw);
// plan + bucketing + k_fill + k_rows over device windows (caller holds ctx->mu);
// sjw != nullptr: splice-junction windows on their segments
int gsnapdp__fill_pipeline(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_window* d_windows, int n,
                           const char* d_query, const char* d_query_uc, gsnapdp_result* d_results,
                           uint32_t* d_ops, const int64_t* d_op_offsets, const gsnapdp_sj_window* sjw);
// allocate the row-lane classes' global scratch on first use
int gsnapdp__rows_pools(gsnapdp_ctx* ctx);
// LDS guard, run once by gsnapdp_create: a kernel's static LDS (hipFuncGetAttributes)
// plus the dynamic LDS it is launched with must fit one workgroup's LDS (max_lds), or
// the launch aborts the queue (HSA_STATUS_ERROR_INVALID_ALLOCATION) instead of
// failing with a message.  Returns -1 with gsnapdp_last_error naming the kernel.
int gsnapdp__lds_fits(const void* fn, size_t dyn, size_t max_lds, const char* name);
int gsnapdp__ggap_lds_check(size_t max_lds);   // gsnapdp_ggap.hip's kernels
int gsnapdp__gband_lds_check(size_t max_lds);  // k_gband
int gsnapdp__micro_lds_check(size_t max_lds);  // k_micro
int gsnapdp__gather_lds_check(size_t max_lds); // k_compact
int gsnapdp__gwin_lds_check(size_t max_lds);   // k_gwin
// k_gband over the register-band lists of a genome-gap batch (gsnapdp_gband.hip)
int gsnapdp__gband_launch(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_ggap_window* d_windows,
                          const int* lists, const int* counts, int list_cap, const char* d_query,
                          const char* d_query_uc, gsnapdp_ggap_result* d_results,
                          gsnapdp_ggap_trace* d_traces, uint32_t* d_ops, const int64_t* d_op_offsets,
                          int use_band);
// k_gwin over the window-per-lane list of a genome-gap batch (gsnapdp_gwin.hip)
int gsnapdp__gwin_launch(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_ggap_window* d_windows,
                         const int* lists, const int* counts, int list_cap, const char* d_query,
                         const char* d_query_uc, gsnapdp_ggap_result* d_results, gsnapdp_ggap_trace* d_traces,
                         uint32_t* d_ops, const int64_t* d_op_offsets);

#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      gsnapdp__set_err(std::string(#x) + ": " + hipGetErrorString(e_));                  \
      return -1;                                                                         \
    }                                                                                    \
  } while (0)

struct gsnapdp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  const uint32_t* h_blocks = nullptr;
  size_t nwords = 0;
  uint32_t* d_blocks = nullptr;
  int mode = 0;
  uint32_t h_prof[gsnapdp::PROF_WORDS];
  uint32_t* d_prof = nullptr;
  double* d_tables = nullptr;
  size_t ntables = 0;
  // per-run scratch
  int cap_n = 0;
  int* d_keys = nullptr;
  int* d_perm = nullptr;
  int* d_big_list = nullptr;
  int* d_small = nullptr;  // hist[NKEYS] | cursor[NKEYS] | class_start[NCLASS+1] | row-lane counts
  size_t perm_cap = 0;
  uint32_t* d_dirpool = nullptr;
  size_t dirpool_waves = 0;
  uint32_t* d_bigpool = nullptr;   // global scratch of the largest row-lane windows (k_rows)
  uint32_t* d_largepool = nullptr; // global scratch of the RW_LARGE row-lane windows
  // host-run staging
  size_t stage_cap = 0;
  void* d_stage = nullptr;
  std::string arch;
  std::mutex mu;
  int fill_waves = 0;  // waves launched per k_fill class kernel
  int fill_stagger = 0;  // k_fill: first traceback batch k * this short in the k-th block of a CU (GSNAPDP_FILL_STAGGER)
  int fill_min_tasks = 0;  // k_fill: fewer waves per SIMD below this many tasks per wave (GSNAPDP_FILL_MIN_TASKS)
  int fill_split = -1;   // k_fill: waves split among the band classes: -1 small batches, 0 never, 1 always (GSNAPDP_FILL_SPLIT)
  int fill_split_w = 5;  // k_fill: a class's per-task weight S + this (GSNAPDP_FILL_SPLIT_W)
  int num_cus = 0;
  // per-stage event timing (gsnapdp_profile)
  int prof_on = 0;
  hipEvent_t ev[2 * 16] = {};
  int ev_used[16] = {};
  // genome-gap batches (gsnapdp_ggap.hip)
  int ggap_cap = 0;
  int* d_ggap_lists = nullptr;     // per-class window lists, GG_NLISTS x ggap_cap
  int* d_ggap_counts = nullptr;    // per-class counts
  uint32_t* d_ggap_pool = nullptr; // global scratch of the large-window path
  uint32_t* d_gband_pool = nullptr; // per-wave scratch of the register-band path (k_gband), score mode
  uint32_t* d_gband_pool_prob = nullptr;  // the same with probability mode's part (first use)
  uint32_t* d_gwin_pool = nullptr;  // per-wave scratch of k_gwin (first use)
  double* d_gwin_probs = nullptr;   // k_gwin_probs' site probabilities, 64 per list window
  size_t gwin_probs_cap = 0;
  int gwin_on = 1;                  // probability-mode windows on k_gwin (GSNAPDP_GWIN=0: off)
  int gwin_min = 16384;             // smallest genome-gap batch on k_gwin (GSNAPDP_GWIN_MIN)
  int ggap_rowlane_only = 0;        // GSNAPDP_GGAP_ROWLANE=1: every window on k_ggap (A/B tests)
  int ggap_use_band = 1;            // k_ggap_plan's GB_USE_* bits (GSNAPDP_GBAND_PROB=1 sets the prob bit)
  int gband_min = 16384;            // smallest genome-gap batch on the register band (GSNAPDP_GBAND_MIN)
  int ends_rowlane = 0;             // GSNAPDP_ENDS_ROWLANE=1: every end gap on k_rows (A/B tests)
  size_t ggap_stage_cap = 0;
  void* d_ggap_stage = nullptr;
  // splice-junction end gaps (gsnapdp_sj_*)
  int sj_cap = 0;
  gsnapdp_window* d_sj_win = nullptr;  // the end-gap records k_sj_plan derives
  // op-stream compaction (gsnapdp_gather.hip): per-block op counts
  int csum_cap = 0;
  int64_t* d_csum = nullptr;    // k_compact: per-block status words (epoch-tagged)
  uint32_t compact_epoch = 0;
  hipEvent_t compact_done = nullptr;  // the last compaction's launch (the next one waits for it)
  // score_introns batches (gsnapdp_score_introns_host): device staging
  size_t si_cap = 0;
  char* d_si_stage = nullptr;
  // host round trips (gsnapdp_run_host): one at a time per context
  std::mutex host_mu;
  void* h_small = nullptr;          // pinned: the compaction header
  void* h_in = nullptr;             // pinned: a small batch's inputs, packed for one H2D copy
  size_t h_in_cap = 0;
  char* d_mx_stage = nullptr;       // gsnapdp_maxent_host: positions in, probabilities out
  size_t mx_cap = 0;
  void* h_mx = nullptr;             // pinned: its packed inputs / outputs
  size_t h_mx_cap = 0;
  std::vector<uint32_t> h_comp;     // compacted ops on their way to op_offsets
  // stage-3 pass executors (gsnapdp_stage3_exec.cpp): staging of idle ones
  std::mutex s3_mu;
  std::vector<void*> s3_pool;
  // traverse_dual_break's stage-2 realignment, served by the caller
  // (gsnapdp_stage3_set_stage2)
  gsnapdp_s3_stage2 s3_stage2 = {nullptr, nullptr};
};
// frees the context's idle stage-3 executors (gsnapdp_destroy)
void gsnapdp__s3_pool_free(gsnapdp_ctx* ctx);

