// gsnapdp_stage3.h -- the stage-3 passes' batch executor (internal).
//
// A pass (gsnapdp_stage3.cpp) advances many paths at once: every round it packs
// the one pending DP window of each waiting path -- single gaps, genome gaps,
// cDNA gaps and microexons -- into ONE input buffer (query bytes, then each
// family's window records and op offsets), and the executor runs the four
// families on it and brings their results back into ONE output buffer.  A pass
// keeps two such rounds in flight (two cohorts of paths, one slot each), so
// the host work of one cohort overlaps the other cohort's batch.
//
// The product executor (gsnapdp_stage3_exec.cpp) stages each slot through
// page-locked memory: one H2D copy, the families' device pipelines back to
// back on the context stream, one D2H copy and an event; the CPU test build
// (tests/dropin/stage3_exec_host.cpp) serves the same layout with the host
// entry points.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>
#include <vector>

#include "../../include/gsnapdp.h"

namespace gsnapdp {

enum S3Fam { S3F_GAP = 0, S3F_GGAP = 1, S3F_CGAP = 2, S3F_MICRO = 3, S3F_N = 4 };

// Byte offsets of one round's regions (each 256-byte aligned).
struct S3Layout {
  int n[S3F_N] = {0, 0, 0, 0};
  size_t q = 0, qu = 0, qbytes = 0;           // in: query, query_uc (qbytes each)
  size_t w[S3F_N] = {0, 0, 0, 0};             // in: window records
  size_t off[S3F_N] = {0, 0, 0, 0};           // in: int64 op offsets, n + 1 each (not for microexons)
  size_t in_bytes = 0;
  size_t r[S3F_N] = {0, 0, 0, 0};             // out: results
  size_t t = 0;                               // out: genome-gap traces
  size_t ops[S3F_N] = {0, 0, 0, 0};           // out: op streams, capacity layout (op offsets)
  size_t out_bytes = 0;
};

class S3Exec {
 public:
  virtual ~S3Exec() {}
  // the slot's input / output staging, at least `bytes` long (contents are not kept)
  virtual char* in_buf(int slot, size_t bytes) = 0;
  virtual char* out_buf(int slot, size_t bytes) = 0;
  // run every family of the slot's packed round; the results are in out_buf(slot)
  // once wait(slot) returns 0.  Returns 0 or -1 (gsnapdp_last_error).
  virtual int submit(int slot, const S3Layout& L) = 0;
  virtual int wait(int slot) = 0;
};

// fn(i) for every i in [0, n) on the passes' persistent host threads (the
// calling thread included); not reentrant (a pass calls it between rounds).
void s3_parallel_for(int n, int grain, const std::function<void(int)>& fn);

// An executor for one pass over `ctx` (2 slots), taken from the context's pool
// (created on first use; concurrent passes each get their own staging) and
// handed back with s3_exec_release.
S3Exec* s3_exec_acquire(gsnapdp_ctx* ctx);
void s3_exec_release(gsnapdp_ctx* ctx, S3Exec* e);

// Driven passes (gsnapdp_stage3_compute): when path i's pass ends, next() gets
// its call (out fields written, status -1 for a failed path) and its list (list
// order, full records, an input pair with the src the driver gave it, a new
// pair with src -1; the driver may take the vector's storage), and returns the
// path's next pass -- its call, and its
// list in *pairs / *n, which must stay valid until that pass ends -- or nullptr
// when the path is finished.  The next pass starts in the same round, so paths
// at different passes share every round's batches.  Called on the pass's host
// threads, each path from one thread at a time.
class S3Driver {
 public:
  virtual ~S3Driver() {}
  virtual gsnapdp_s3_call* next(int i, gsnapdp_s3_call* ended, std::vector<gsnapdp_s3_pair>& list,
                                const gsnapdp_s3_pair** pairs, int* n) = 0;
};
// the pass over the calls' first passes, every path continued by the driver;
// no lists are written (the driver has them)
int s3_run_driven(gsnapdp_ctx* ctx, gsnapdp_s3_call* calls, int ncalls, const gsnapdp_s3_pair* pairs_in,
                  int64_t npairs_in, const char* query, const char* query_uc, size_t query_bytes,
                  const gsnapdp_iit* iit, S3Driver* driver, gsnapdp_s3_stats* stats);

// get_genomic_nt (stage3.c) on the packed genome, with no genomic segment: the
// character at position gpos of the call's genomic stretch, '*' outside it
char s3_genomic_nt(const uint32_t* blocks, size_t nwords, const gsnapdp_s3_call& c, int gpos);

// the context's stage-2 callback for traverse_dual_break (gsnapdp_stage3_set_stage2)
gsnapdp_s3_stage2 s3_stage2(gsnapdp_ctx* ctx);
void s3_set_stage2(gsnapdp_ctx* ctx, const gsnapdp_s3_stage2& s2);

}  // namespace gsnapdp
