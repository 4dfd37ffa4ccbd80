// gsnapdp_dropin.cpp -- the reference's per-call entry points (include/
// gsnapdp_dropin.h) over the batched C-ABI of include/gsnapdp.h.
//
// Each gap-filler call becomes a batch of one window: the query bytes the
// reference would read are staged, the GPU runs fill + endpoint + traceback,
// and the op stream is expanded into pairs that are pushed into the caller's
// Pairpool so that the returned List_T is the reference's, cell for cell.
// There is no CPU fallback: without a gfx950 device the first call aborts,
// as the reference aborts on its own fatal conditions.
#include <dlfcn.h>
#include <stddef.h>
#include <malloc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <utility>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gsnapdp.h"
#include "../../include/gsnapdp_dropin.h"
#include "gsnapdp_internal.h"
#include "gsnapdp_pairlayout.h"

namespace {

struct Dynprog {  // the Dynprog_T workspace: only its length limits matter here
  int maxlength1, maxlength2;
};

struct State {
  std::mutex mu;
  int mode = 0;
  const unsigned int* blocks = nullptr;
  size_t nwords = 0;
  int device = 0;
  bool explicit_genome = false;  // Gsnapdp_dropin_genome was called
  gsnapdp_ctx* ctx = nullptr;
  bool tables = false;
  bool splicing_iit = false;  // Dynprog_setup got known splice sites
  // the splicing IIT itself and how Dynprog_setup described it (dynprog.c:350-376)
  gsnapdp_IIT_T iit = nullptr;
  int* divint_crosstable = nullptr;
  int donor_typeint = -1, acceptor_typeint = -1;
  bool novelsplicingp = true;
  // known splice sites and their tries (Dynprog_setup, dynprog.c:350-376)
  const unsigned* splicesites = nullptr;
  const int* splicetypes = nullptr;
  int nsplicesites = 0;
  unsigned *trieoffsets_obs = nullptr, *triecontents_obs = nullptr;
  unsigned *trieoffsets_max = nullptr, *triecontents_max = nullptr;
};
State g;


[[noreturn]] void fatal(const std::string& msg) {
  fprintf(stderr, "gsnapdp drop-in: %s\n", msg.c_str());
  abort();
}

// Context on first use.  The genome comes from the host program's own setup
// calls, so gmap / gsnap link the library unchanged:
//  * index genome: Dynprog_setup's Genome_T (gmap.c:3828, gsnap.c:2366) gives
//    Genome_blocks / Genome_totallength (genome.c:96-107), resolved in the host;
//  * user segment (gmap -g): Dynprog_setup gets NULL and the blocks arrive in
//    Maxent_hr_setup (gmap.c:3803) from Genome_create_blocks, a CALLOC of
//    ((len+31)/32)*3 + 4 words (genome-write.c:809-810); the allocation's
//    usable size covers every block the DP can address.
// Gsnapdp_dropin_genome(blocks, nwords, device) still overrides both.
gsnapdp_ctx* ctx() {
  if (g.ctx) return g.ctx;
  if (!g.blocks) fatal("no genome: neither Dynprog_setup nor Maxent_hr_setup gave the genome blocks");
  if (!g.nwords) g.nwords = malloc_usable_size((void*)g.blocks) / sizeof(unsigned int);
  if (!g.nwords) fatal("cannot size the genome blocks; call Gsnapdp_dropin_genome(blocks, nwords, device)");
  g.ctx = gsnapdp_create(g.device, g.blocks, g.nwords, g.mode);
  if (!g.ctx) fatal(std::string("gsnapdp_create: ") + gsnapdp_last_error());
  return g.ctx;
}

// MaxEnt tables: $GSNAPDP_MAXENT_TABLES, else <libdir>/../data/maxent_hr_tables.bin
void ensure_tables() {
  if (g.tables) return;
  std::string path;
  if (const char* e = getenv("GSNAPDP_MAXENT_TABLES")) {
    path = e;
  } else {
    Dl_info info;
    if (dladdr((void*)&ensure_tables, &info) && info.dli_fname) {
      path = info.dli_fname;
      path = path.substr(0, path.rfind('/')) + "/../data/maxent_hr_tables.bin";
    }
  }
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) fatal("cannot open MaxEnt tables " + path);
  std::vector<double> t(12 * 16384 + 4 * 16);
  const size_t n = fread(t.data(), sizeof(double), t.size(), f);
  fclose(f);
  if (n != t.size()) fatal("short MaxEnt table file " + path);
  if (gsnapdp_load_maxent_tables(ctx(), t.data(), t.size()))
    fatal(std::string("load tables: ") + gsnapdp_last_error());
  g.tables = true;
}

// ---- windows from concurrent callers, combined into batches
// gmap / gsnap call the Dynprog_* / Maxent_hr_* entry points synchronously
// from each worker thread (gmap -t N).  A caller queues its request (one
// window of any family, or one MaxEnt position); whichever caller finds no
// batch in flight becomes the leader, takes every queued request, runs one
// batch per family through the batched C-ABI (page-locked staging) and wakes
// the owners, which expand their own op streams into their own Pairpools.
// No global lock is held across a GPU round trip; one thread alone sees
// batches of one.
enum Fam { F_GAP, F_GGAP, F_CGAP, F_SJ, F_MICRO, F_MAXENT, F_INTRONS, F_N };

struct Req {
  int fam;
  bool done = false;
  std::vector<char> q, qu;  // this window's query bytes; positions in w are relative to them
  int64_t cap = 0;          // op capacity
  std::vector<uint32_t> ops;
  explicit Req(int f) : fam(f) {}
};
struct GapReq : Req {
  gsnapdp_window w;
  gsnapdp_result r;
  GapReq() : Req(F_GAP) {}
};
struct GgapReq : Req {
  gsnapdp_ggap_window w;
  gsnapdp_ggap_result r;
  gsnapdp_ggap_trace t;
  GgapReq() : Req(F_GGAP) {}
};
struct CgapReq : Req {
  gsnapdp_cgap_window w;
  gsnapdp_cgap_result r;
  CgapReq() : Req(F_CGAP) {}
};
struct SjReq : Req {
  gsnapdp_sj_window w;
  gsnapdp_result r;
  SjReq() : Req(F_SJ) {}
};
struct MicroReq : Req {
  gsnapdp_micro_window w;
  gsnapdp_micro_result r;
  MicroReq() : Req(F_MICRO) {}
};
struct MaxReq : Req {
  uint8_t model;
  unsigned pos, chroffset;
  double out = 0.0;
  MaxReq() : Req(F_MAXENT) {}
};
struct IntronReq : Req {  // one score_introns path
  gsnapdp_intron_path p;
  std::vector<gsnapdp_intron> introns;
  gsnapdp_intron_scores out;
  IntronReq() : Req(F_INTRONS) {}
};

// Page-locked host arrays of the leader's batches (gsnapdp_host_alloc), grown
// geometrically and kept for the life of the process.
template <class T>
struct Pinned {
  T* p = nullptr;
  size_t cap = 0;
  T* get(size_t n) {
    if (n > cap) {
      if (p) gsnapdp_host_free(p);
      cap = n + n / 2 + 64;
      p = (T*)gsnapdp_host_alloc(cap * sizeof(T));
      if (!p) fatal(std::string("page-locked staging: ") + gsnapdp_last_error());
    }
    return p;
  }
};

struct Batcher {
  std::mutex m;
  std::condition_variable cv;
  std::vector<Req*> pending;
  bool busy = false;
  unsigned long batches[F_N] = {}, maxbatch[F_N] = {}, windows[F_N] = {};
  double gpu_s[F_N] = {};  // leader time in each family's batched round trip
  // leader-only staging
  Pinned<char> Q, QU;
  Pinned<int64_t> OFF;
  Pinned<uint32_t> OPS;
  Pinned<unsigned char> W, R, T;
};
Batcher gb;

struct StatsAtExit {
  ~StatsAtExit() {
    if (!getenv("GSNAPDP_DROPIN_STATS")) return;
    static const char* names[F_N] = {"gap", "genome_gap", "cdna_gap", "splicejunction", "microexon",
                                     "maxent", "score_introns"};
    fprintf(stderr, "gsnapdp_dropin:");
    for (int f = 0; f < F_N; f++)
      fprintf(stderr, " %s %lu in %lu batches (largest %lu, %.3f s);", names[f], gb.windows[f],
              gb.batches[f], gb.maxbatch[f], gb.gpu_s[f]);
    fprintf(stderr, "\n");
  }
} stats_at_exit;

// Concatenates the requests' query bytes and op ranges into the staging
// arrays; returns each request's query offset.
template <class X>
std::vector<size_t> pack(const std::vector<X*>& b, size_t* qbytes) {
  size_t qn = 0;
  for (const X* x : b) qn += x->q.size();
  char* Q = gb.Q.get(qn + 8);
  char* QU = gb.QU.get(qn + 8);
  int64_t* OFF = gb.OFF.get(b.size() + 1);
  std::vector<size_t> qo(b.size());
  size_t o = 0;
  OFF[0] = 0;
  for (size_t i = 0; i < b.size(); i++) {
    memcpy(Q + o, b[i]->q.data(), b[i]->q.size());
    memcpy(QU + o, b[i]->qu.data(), b[i]->qu.size());
    qo[i] = o;
    o += b[i]->q.size();
    OFF[i + 1] = OFF[i] + b[i]->cap;
  }
  gb.OPS.get((size_t)OFF[b.size()] + 1);
  *qbytes = o;
  return qo;
}
template <class X>
void unpack_ops(const std::vector<X*>& b) {
  const int64_t* OFF = gb.OFF.p;
  for (size_t i = 0; i < b.size(); i++) b[i]->ops.assign(gb.OPS.p + OFF[i], gb.OPS.p + OFF[i + 1]);
}
template <class Win>
Win* windows_of(size_t n) { return (Win*)gb.W.get(n * sizeof(Win)); }
template <class Res>
Res* results_of(size_t n) { return (Res*)gb.R.get(n * sizeof(Res)); }

void check(int rc, const char* what) {
  if (rc) fatal(std::string(what) + ": " + gsnapdp_last_error());
}

// the leader, without gb.m held: one batch per family
void run_family(gsnapdp_ctx* c, int fam, std::vector<Req*>& reqs) {
  const size_t n = reqs.size();
  size_t qb = 0;
  switch (fam) {
    case F_GAP: {
      std::vector<GapReq*> b;
      for (Req* r : reqs) b.push_back((GapReq*)r);
      const std::vector<size_t> qo = pack(b, &qb);
      gsnapdp_window* W = windows_of<gsnapdp_window>(n);
      gsnapdp_result* R = results_of<gsnapdp_result>(n);
      for (size_t i = 0; i < n; i++) {
        W[i] = b[i]->w;
        W[i].qpos += (uint32_t)qo[i];
      }
      check(gsnapdp_run_host(c, W, (int)n, gb.Q.p, gb.QU.p, qb, R, gb.OPS.p, gb.OFF.p), "gsnapdp_run_host");
      for (size_t i = 0; i < n; i++) b[i]->r = R[i];
      unpack_ops(b);
      break;
    }
    case F_GGAP: {
      std::vector<GgapReq*> b;
      for (Req* r : reqs) b.push_back((GgapReq*)r);
      const std::vector<size_t> qo = pack(b, &qb);
      gsnapdp_ggap_window* W = windows_of<gsnapdp_ggap_window>(n);
      gsnapdp_ggap_result* R = results_of<gsnapdp_ggap_result>(n);
      gsnapdp_ggap_trace* T = (gsnapdp_ggap_trace*)gb.T.get(n * sizeof(gsnapdp_ggap_trace));
      for (size_t i = 0; i < n; i++) {
        W[i] = b[i]->w;
        W[i].qpos += (uint32_t)qo[i];
      }
      check(gsnapdp_ggap_run_host(c, W, (int)n, gb.Q.p, gb.QU.p, qb, R, T, gb.OPS.p, gb.OFF.p),
            "gsnapdp_ggap_run_host");
      for (size_t i = 0; i < n; i++) {
        b[i]->r = R[i];
        b[i]->t = T[i];
      }
      unpack_ops(b);
      break;
    }
    case F_CGAP: {
      std::vector<CgapReq*> b;
      for (Req* r : reqs) b.push_back((CgapReq*)r);
      const std::vector<size_t> qo = pack(b, &qb);
      gsnapdp_cgap_window* W = windows_of<gsnapdp_cgap_window>(n);
      gsnapdp_cgap_result* R = results_of<gsnapdp_cgap_result>(n);
      for (size_t i = 0; i < n; i++) {
        W[i] = b[i]->w;
        W[i].qposL += (uint32_t)qo[i];
        W[i].qposR += (uint32_t)qo[i];
      }
      check(gsnapdp_cgap_run_host(c, W, (int)n, gb.Q.p, gb.QU.p, qb, R, gb.OPS.p, gb.OFF.p),
            "gsnapdp_cgap_run_host");
      for (size_t i = 0; i < n; i++) b[i]->r = R[i];
      unpack_ops(b);
      break;
    }
    case F_SJ: {
      std::vector<SjReq*> b;
      for (Req* r : reqs) b.push_back((SjReq*)r);
      const std::vector<size_t> qo = pack(b, &qb);
      gsnapdp_sj_window* W = windows_of<gsnapdp_sj_window>(n);
      gsnapdp_result* R = results_of<gsnapdp_result>(n);
      for (size_t i = 0; i < n; i++) {
        W[i] = b[i]->w;
        W[i].qpos += (uint32_t)qo[i];
        W[i].spos += (uint32_t)qo[i];
      }
      check(gsnapdp_sj_run_host(c, W, (int)n, gb.Q.p, gb.QU.p, qb, R, gb.OPS.p, gb.OFF.p),
            "gsnapdp_sj_run_host");
      for (size_t i = 0; i < n; i++) b[i]->r = R[i];
      unpack_ops(b);
      break;
    }
    case F_MICRO: {
      std::vector<MicroReq*> b;
      for (Req* r : reqs) b.push_back((MicroReq*)r);
      const std::vector<size_t> qo = pack(b, &qb);
      gsnapdp_micro_window* W = windows_of<gsnapdp_micro_window>(n);
      gsnapdp_micro_result* R = results_of<gsnapdp_micro_result>(n);
      for (size_t i = 0; i < n; i++) {
        W[i] = b[i]->w;
        W[i].qpos += (uint32_t)qo[i];
        W[i].ppos += (uint32_t)qo[i];
      }
      check(gsnapdp_micro_run_host(c, W, (int)n, gb.Q.p, gb.QU.p, qb, R), "gsnapdp_micro_run_host");
      for (size_t i = 0; i < n; i++) b[i]->r = R[i];
      break;
    }
    case F_MAXENT: {
      uint8_t* M = (uint8_t*)gb.Q.get(n + 8);
      unsigned* P = (unsigned*)gb.W.get(2 * n * sizeof(unsigned));
      double* O = (double*)gb.R.get(n * sizeof(double));
      for (size_t i = 0; i < n; i++) {
        const MaxReq* x = (const MaxReq*)reqs[i];
        M[i] = x->model;
        P[i] = x->pos;
        P[n + i] = x->chroffset;
      }
      check(gsnapdp_maxent_host(c, M, P, P + n, O, (int)n), "maxent");
      for (size_t i = 0; i < n; i++) ((MaxReq*)reqs[i])->out = O[i];
      break;
    }
    case F_INTRONS: {  // every queued path in one k_introns launch
      std::vector<gsnapdp_intron_path> P(n);
      std::vector<gsnapdp_intron> I;
      for (size_t i = 0; i < n; i++) {
        IntronReq* x = (IntronReq*)reqs[i];
        P[i] = x->p;
        P[i].first_intron = (int32_t)I.size();
        P[i].nintrons = (int32_t)x->introns.size();
        for (gsnapdp_intron t : x->introns) {
          t.path = (int32_t)i;
          I.push_back(t);
        }
      }
      std::vector<gsnapdp_intron_scores> O(n);
      check(gsnapdp_score_introns_host(c, P.data(), (int)n, I.data(), (int)I.size(), O.data()),
            "gsnapdp_score_introns_host");
      for (size_t i = 0; i < n; i++) ((IntronReq*)reqs[i])->out = O[i];
      break;
    }
  }
}

// Queue `r` and return once its batch ran (this thread may be the leader).
void submit(gsnapdp_ctx* c, Req* r) {
  std::unique_lock<std::mutex> lk(gb.m);
  gb.pending.push_back(r);
  while (!r->done) {
    if (!gb.busy) {
      gb.busy = true;
      std::vector<Req*> batch;
      batch.swap(gb.pending);
      lk.unlock();
      std::vector<Req*> fam[F_N];
      for (Req* x : batch) fam[x->fam].push_back(x);
      double dt[F_N] = {};
      for (int f = 0; f < F_N; f++) {
        if (fam[f].empty()) continue;
        const auto t0 = std::chrono::steady_clock::now();
        run_family(c, f, fam[f]);
        dt[f] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      }
      lk.lock();
      for (int f = 0; f < F_N; f++) {
        if (fam[f].empty()) continue;
        gb.gpu_s[f] += dt[f];
        gb.batches[f]++;
        gb.windows[f] += fam[f].size();
        if (fam[f].size() > gb.maxbatch[f]) gb.maxbatch[f] = fam[f].size();
      }
      for (Req* x : batch) x->done = true;
      gb.busy = false;
      gb.cv.notify_all();
    } else {
      gb.cv.wait(lk);
    }
  }
}

gsnapdp_ctx* shared_ctx(bool tables) {
  std::lock_guard<std::mutex> lock(g.mu);
  if (tables) ensure_tables();
  return ctx();
}

// pushes a pair list (final order) into the caller's pool, last pair first
// (gapp bit 1: a knownp gapholder)
gsnapdp_List_T push_pairs(const gsnapdp_pair* pairs, int n, gsnapdp_Pairpool_T pool) {
  gsnapdp_List_T list = nullptr;
  for (int i = n - 1; i >= 0; i--) {
    const gsnapdp_pair& p = pairs[i];
    if (p.gapp)
      list = Pairpool_push_gapholder(list, pool, p.queryjump, p.genomejump, (p.gapp & 2) ? 1 : 0);
    else
      list = Pairpool_push(list, pool, p.querypos, p.genomepos, p.cdna, p.comp, p.genome,
                           p.dynprogindex);
  }
  return list;
}

gsnapdp_List_T run_one(gsnapdp_window& w, const char* seq, const char* sequc, bool rev,
                       gsnapdp_Pairpool_T pool, int* dynprogindex, int* finalscore,
                       int* nmatches, int* nmismatches, int* nopens, int* nindels) {
  gsnapdp_ctx* c = shared_ctx(false);
  GapReq req;
  const int L1 = w.length1 > 0 ? w.length1 : 0;
  // query bytes the reference may read: sequence1[0..L1) or revsequence1[-(L1-1)..0],
  // padded to a 4-byte multiple (the kernels read dwords)
  const size_t qsz = ((size_t)L1 + 8 + 3) & ~(size_t)3;
  req.q.assign(qsz, 0);
  req.qu.assign(qsz, 0);
  if (L1 > 0) {
    memcpy(req.q.data(), rev ? seq - (L1 - 1) : seq, (size_t)L1);
    memcpy(req.qu.data(), rev ? sequc - (L1 - 1) : sequc, (size_t)L1);
  }
  w.qpos = rev ? (uint32_t)(L1 > 0 ? L1 - 1 : 0) : 0u;
  req.w = w;
  req.cap = (int64_t)L1 + (w.length2 > 0 ? w.length2 : 0) + 2;
  submit(c, &req);
  const gsnapdp_result& r = req.r;
  if (r.status == gsnapdp::ST_UNSUPPORTED)
    fatal("window outside the reference's domain (the reference aborts here)");
  if (r.status == gsnapdp::ST_OPS_OVERFLOW) fatal("op stream overflow");
  thread_local std::vector<gsnapdp_pair> pairs;
  pairs.resize((size_t)req.cap + 8);
  int fs = 0;
  const int n = gsnapdp_expand(c, &w, &r, req.ops.data(), req.q.data(), req.qu.data(), pairs.data(),
                               (int)pairs.size(), &fs);
  if (n < 0 || n > (int)pairs.size()) fatal("gsnapdp_expand failed");
  *dynprogindex = r.reserved;  // the stepped *dynprogindex
  *finalscore = r.finalscore;
  *nmatches = r.nmatches;
  *nmismatches = r.nmismatches;
  *nopens = r.nopens;
  *nindels = r.nindels;
  return push_pairs(pairs.data(), n, pool);
}

gsnapdp_window base_window(int kind, int length1, int length2, int offset1, int offset2,
                           unsigned chroffset, unsigned chrhigh, unsigned chrpos,
                           unsigned genomiclength, int cdna_direction, int watsonp,
                           int jump_late_p, int extraband, double defect_rate,
                           const Dynprog* dp, int dynprogindex) {
  gsnapdp_window w;
  memset(&w, 0, sizeof(w));
  w.kind = kind;
  w.length1 = length1;
  w.length2 = length2;
  w.offset1 = offset1;
  w.offset2 = offset2;
  w.chroffset = chroffset;
  w.chrhigh = chrhigh;
  w.chrpos = chrpos;
  w.genomiclength = genomiclength;
  w.cdna_direction = cdna_direction;
  w.extraband = extraband;
  w.dynprogindex = dynprogindex;
  w.maxlength1 = dp->maxlength1;
  w.maxlength2 = dp->maxlength2;
  // only the bin matters (dynprog.c:4471-4486): keep the double comparison exact
  w.defect_rate = defect_rate < 0.003 ? 0.001f : (defect_rate < 0.014 ? 0.01f : 0.5f);
  w.watsonp = watsonp ? 1 : 0;
  w.jump_late_p = jump_late_p ? 1 : 0;
  return w;
}

double maxent_one(int model, unsigned splice_pos, unsigned chroffset) {
  gsnapdp_ctx* c = shared_ctx(true);
  MaxReq req;
  req.model = (uint8_t)model;
  req.pos = splice_pos;
  req.chroffset = chroffset;
  submit(c, &req);
  return req.out;
}

// Genome_fill_buffer_blocks_noterm (genome.c:10090) on the host copy of the
// blocks: uncompress_mmap (genome.c:8912) writes "ACGT"[2 bits], 'N' where the
// flag bit is set.  (Host staging of the caller's splice junction, like the
// reference's; the DP on it runs on the GPU.)
void fill_buffer(unsigned left, unsigned length, char* out) {
  if (!g.blocks) fatal("no genome: call Gsnapdp_dropin_genome before Dynprog_make_splicejunction_*");
  for (unsigned i = 0; i < length; i++) {
    const unsigned pos = left + i;
    const size_t ptr = (size_t)(pos >> 5) * 3;
    if (ptr + 2 >= g.nwords) fatal("junction outside the genome");
    const unsigned bit = pos & 31u;
    if ((g.blocks[ptr + 2] >> bit) & 1u) {
      out[i] = 'N';
    } else {
      const unsigned word = bit < 16 ? g.blocks[ptr + 1] : g.blocks[ptr];
      out[i] = "ACGT"[(word >> ((bit & 15u) * 2u)) & 3u];
    }
  }
}

// make_complement_inplace (dynprog.c:1392-1406): reverse complement with
// complCode = COMPLEMENT_LC (complement.h:31)
void revcomp_inplace(char* s, int length) {
  static const char* lc =
      "???????????????????????????????? ??#$%&')(*+,-./0123456789:;>=<??TVGHEFCDIJMLKNOPQYSAABWXRZ]?"
      "[^_`tvghefcdijmlknopqysaabwxrz}|{~?";
  auto cc = [&](char c) { return lc[(unsigned char)c & 127u]; };
  if (length <= 0) return;
  int i = 0, j = length - 1;
  for (; i < length / 2; i++, j--) {
    const char t = cc(s[i]);
    s[i] = cc(s[j]);
    s[j] = t;
  }
  if (i == j) s[i] = cc(s[i]);
}

enum { DONOR = 0, ANTIDONOR = 1, ACCEPTOR = 2, ANTIACCEPTOR = 3 };  // splicetrie_build.h:4

// Dynprog_end5/3_splicejunction as a batch of one (gsnapdp_sj_*).
gsnapdp_List_T run_sj(int kind, const char* seq1, const char* seq1uc, const char* seq2,
                      const char* seq2uc, int length1, int length2, int offset1, int anchor,
                      int far, int contlength, int cdna_direction, int watsonp, int jump_late_p,
                      int extraband_end, double defect_rate, const Dynprog* dp,
                      gsnapdp_Pairpool_T pool, int* dynprogindex, int* finalscore, int* nmatches,
                      int* nmismatches, int* nopens, int* nindels) {
  gsnapdp_ctx* c = shared_ctx(false);
  SjReq req;
  gsnapdp_sj_window& w = req.w;
  const bool rev = kind == GSNAPDP_END5_GAP;
  const int L1 = length1 > 0 ? length1 : 0, L2 = length2 > 0 ? length2 : 0;
  memset(&w, 0, sizeof(w));
  w.kind = kind;
  w.length1 = length1;
  w.length2 = length2;
  w.offset1 = offset1;
  w.offset2_anchor = anchor;
  w.offset2_far = far;
  w.contlength = contlength;
  w.cdna_direction = cdna_direction;
  w.extraband_end = extraband_end;
  w.dynprogindex = *dynprogindex;
  w.maxlength1 = dp->maxlength1;
  w.maxlength2 = dp->maxlength2;
  w.defect_rate = defect_rate < 0.003 ? 0.001f : (defect_rate < 0.014 ? 0.01f : 0.5f);
  w.watsonp = watsonp ? 1 : 0;
  w.jump_late_p = jump_late_p ? 1 : 0;
  // query rows then the junction, each with 4 bytes of slack
  const bool run = L1 > 0 && L2 > 0 && L1 <= dp->maxlength1 && L2 <= dp->maxlength2;
  const size_t sbase = (size_t)L1 + 4;
  req.q.assign((sbase + L2 + 8 + 3) & ~(size_t)3, 0);
  req.qu.assign(req.q.size(), 0);
  if (run) {
    memcpy(req.q.data(), rev ? seq1 - (L1 - 1) : seq1, (size_t)L1);
    memcpy(req.qu.data(), rev ? seq1uc - (L1 - 1) : seq1uc, (size_t)L1);
    memcpy(req.q.data() + sbase, rev ? seq2 - (L2 - 1) : seq2, (size_t)L2);
    memcpy(req.qu.data() + sbase, rev ? seq2uc - (L2 - 1) : seq2uc, (size_t)L2);
  }
  w.qpos = rev ? (uint32_t)(L1 > 0 ? L1 - 1 : 0) : 0u;
  w.spos = (uint32_t)(rev ? sbase + (L2 > 0 ? L2 - 1 : 0) : sbase);
  const int64_t cap = (int64_t)L1 + L2 + 2;
  req.cap = cap;
  submit(c, &req);
  const gsnapdp_result& r = req.r;
  if (r.status == gsnapdp::ST_UNSUPPORTED) fatal("splice junction outside A C G T N");
  if (r.status == gsnapdp::ST_OPS_OVERFLOW) fatal("op stream overflow");
  *nmatches = r.nmatches;
  *nmismatches = r.nmismatches;
  *nopens = r.nopens;
  *nindels = r.nindels;
  *finalscore = r.finalscore;
  *dynprogindex = r.reserved;
  if (r.status == gsnapdp::ST_EARLY) return nullptr;
  thread_local std::vector<gsnapdp_pair> pairs;
  pairs.resize((size_t)cap + 8);
  const int n = gsnapdp_sj_expand(c, &w, &r, req.ops.data(), req.q.data(), req.qu.data(), pairs.data(),
                                  (int)pairs.size());
  if (n < 0 || n > (int)pairs.size()) fatal("gsnapdp_sj_expand failed");
  return push_pairs(pairs.data(), n, pool);
}

// The head of the reference's Pair_T (pairdef.h:9-23) and List_T (listdef.h):
// make_microexon_pairs_double writes the gapholders' comp in place
// (dynprog.c:6990-6991), so the shim does the same through the host's layout.
struct RefPairHead {
  int querypos;
  unsigned genomepos;
  int refquerypos, aapos, queryjump, genomejump, aaphase_g, aaphase_e, dynprogindex;
  char cdna, comp, genome;
};
struct RefList {
  void* first;
  RefList* rest;
};
// ... through the fields score_introns reads (pairdef.h:9-32; flat, so the
// chars and bools pack exactly as in Pair_T)
struct RefPairGap {
  int querypos;
  unsigned genomepos;
  int refquerypos, aapos, queryjump, genomejump, aaphase_g, aaphase_e, dynprogindex;
  char cdna, comp, genome, aa_g, aa_e;
  unsigned char gapp, knowngapp;  // bool (bool.h: unsigned char)
};
static_assert(offsetof(RefPairGap, gapp) == GSNAPDP_PAIR_OFF_GAPP &&
                  offsetof(RefPairGap, knowngapp) == GSNAPDP_PAIR_OFF_KNOWNGAPP,
              "Pair_T layout");
// ... and the whole struct (pairdef.h:9-49), for build_pairs_introns' disallowedp
struct RefPair {
  int querypos;
  unsigned genomepos;
  int refquerypos, aapos, queryjump, genomejump, aaphase_g, aaphase_e, dynprogindex;
  char cdna, comp, genome, aa_g, aa_e;
  unsigned char gapp, knowngapp, extraexonp, shortexonp;
  int state, vstate_good, vstate_bad;  // State_T
  unsigned char protectedp, disallowedp;
  double donor_prob, acceptor_prob;
  unsigned char end_intron_p;
};
// every field the shim touches, against the constants oracle/pairdef_check.c
// asserts against the reference's pairdef.h / listdef.h (gsnapdp_pairlayout.h)
static_assert(offsetof(RefPair, querypos) == GSNAPDP_PAIR_OFF_QUERYPOS &&
                  offsetof(RefPair, genomepos) == GSNAPDP_PAIR_OFF_GENOMEPOS &&
                  offsetof(RefPair, queryjump) == GSNAPDP_PAIR_OFF_QUERYJUMP &&
                  offsetof(RefPair, genomejump) == GSNAPDP_PAIR_OFF_GENOMEJUMP &&
                  offsetof(RefPair, dynprogindex) == GSNAPDP_PAIR_OFF_DYNPROGINDEX &&
                  offsetof(RefPair, cdna) == GSNAPDP_PAIR_OFF_CDNA && offsetof(RefPair, comp) == GSNAPDP_PAIR_OFF_COMP &&
                  offsetof(RefPair, genome) == GSNAPDP_PAIR_OFF_GENOME &&
                  offsetof(RefPair, gapp) == GSNAPDP_PAIR_OFF_GAPP &&
                  offsetof(RefPair, knowngapp) == GSNAPDP_PAIR_OFF_KNOWNGAPP &&
                  offsetof(RefPair, disallowedp) == GSNAPDP_PAIR_OFF_DISALLOWEDP &&
                  offsetof(RefPair, donor_prob) == GSNAPDP_PAIR_OFF_DONOR_PROB &&
                  offsetof(RefPair, shortexonp) == GSNAPDP_PAIR_OFF_SHORTEXONP &&
                  offsetof(RefPair, end_intron_p) == GSNAPDP_PAIR_OFF_END_INTRON_P && sizeof(RefPair) == GSNAPDP_PAIR_SIZE,
              "Pair_T layout");
static_assert(offsetof(RefPairHead, querypos) == GSNAPDP_PAIR_OFF_QUERYPOS &&
                  offsetof(RefPairHead, comp) == GSNAPDP_PAIR_OFF_COMP,
              "Pair_T layout");
static_assert(offsetof(RefList, first) == GSNAPDP_LIST_OFF_FIRST && offsetof(RefList, rest) == GSNAPDP_LIST_OFF_REST &&
                  sizeof(RefList) == GSNAPDP_LIST_SIZE,
              "List_T layout");

// binary_search (dynprog.c:5068-5090)
int binary_search(int lowi, int highi, const unsigned* positions, unsigned goal) {
  while (lowi < highi) {
    const int middlei = (lowi + highi) / 2;
    if (goal < positions[middlei]) highi = middlei;
    else if (goal > positions[middlei]) lowi = middlei + 1;
    else return middlei;
  }
  return highi;
}

// The host program's Splicetrie_solve_end5/3 (splicetrie.c:881, 953).  Weak
// references: a gmap/gsnap link binds them to its splicetrie.o; a host that
// loads the shim before its splicetrie code (dlopen) is served by a lookup at
// the first call.  Without either, the known-site ends fail loudly.
extern "C" __attribute__((weak)) gsnapdp_List_T Splicetrie_solve_end5(
    gsnapdp_List_T, unsigned int*, unsigned int*, int, gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T,
    int*, int*, int*, int*, int*, gsnapdp_bool*, int*, int*, int, int, gsnapdp_Genomicpos_T, char*,
    int, int, gsnapdp_Splicetype_T, gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T,
    int, int*, gsnapdp_Dynprog_T, char*, char*, int, int, int, int, int, gsnapdp_bool, gsnapdp_bool,
    gsnapdp_Pairpool_T, int, double);
extern "C" __attribute__((weak)) gsnapdp_List_T Splicetrie_solve_end3(
    gsnapdp_List_T, unsigned int*, unsigned int*, int, gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T,
    int*, int*, int*, int*, int*, gsnapdp_bool*, int*, int*, int, int, gsnapdp_Genomicpos_T, char*,
    int, int, gsnapdp_Splicetype_T, gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T,
    int, int*, gsnapdp_Dynprog_T, char*, char*, int, int, int, int, int, gsnapdp_bool, gsnapdp_bool,
    gsnapdp_Pairpool_T, int, double);
using SolveFn = decltype(&Splicetrie_solve_end5);

// The host program's genome accessors (genome.c:96-107), for Dynprog_setup.
// The host program's stage 2 (stage2.c:4260), which traverse_dual_break calls
// (stage3.c:7104-7117) for a dual break no single gap can solve
extern "C" __attribute__((weak)) gsnapdp_List_T Stage2_compute_one(
    int* stage2_source, int* stage2_indexsize, char* queryseq_ptr, char* queryuc_ptr, int querylength,
    int query_offset, char* genomicseg_ptr, char* genomicuc_ptr, gsnapdp_Genomicpos_T genomicstart,
    gsnapdp_Genomicpos_T genomicend, gsnapdp_Genomicpos_T mappingstart, gsnapdp_Genomicpos_T mappingend,
    gsnapdp_bool plusp, int genestrand, int genomiclength, void* oligoindices, int noligoindices,
    double proceed_pctcoverage, gsnapdp_Pairpool_T pairpool, void* diagpool, int sufflookback, int nsufflookback,
    int maxintronlen, gsnapdp_bool localp, gsnapdp_bool skip_repetitive_p, gsnapdp_bool use_shifted_canonical_p,
    gsnapdp_bool favor_right_p, gsnapdp_bool debug_graphic_p, gsnapdp_bool diagnosticp, void* stopwatch,
    gsnapdp_bool diag_debug);

extern "C" __attribute__((weak)) unsigned int* Genome_blocks(gsnapdp_Genome_T);
extern "C" __attribute__((weak)) gsnapdp_Genomicpos_T Genome_totallength(gsnapdp_Genome_T);

// The host program's splicing-IIT queries (iit-read.c:3770, 3808, 3973, 4011),
// used exactly where bridge_intron_gap makes them (dynprog.c:3375-3550, 3598-3612).
extern "C" __attribute__((weak)) gsnapdp_bool IIT_exists_with_divno_typed_signed(
    gsnapdp_IIT_T, int divno, unsigned int x, unsigned int y, int type, int sign);
extern "C" __attribute__((weak)) gsnapdp_bool IIT_low_exists_signed_p(gsnapdp_IIT_T, int divno,
                                                                      unsigned int x, int sign);
extern "C" __attribute__((weak)) gsnapdp_bool IIT_high_exists_signed_p(gsnapdp_IIT_T, int divno,
                                                                       unsigned int x, int sign);
extern "C" __attribute__((weak)) gsnapdp_bool IIT_exists_with_divno_signed(
    gsnapdp_IIT_T, int divno, unsigned int x, unsigned int y, int sign);

// The host program's splicing IIT as the batched ABI asks it (gsnapdp_iit):
// each query goes to the host's own iit-read function with the division and
// type ints Dynprog_setup was given (dynprog.c:350-376), so the known-site
// records (gsnapdp_known_site_record) and score_introns' verdicts
// (gsnapdp_introns_known) see exactly what the reference's queries see.
template <class F>
F resolve_host(F f, const char* name) {  // weak reference, else a lookup in the process
  if (!f) f = (F)dlsym(RTLD_DEFAULT, name);
  if (!f) fatal(std::string("the host program's ") + name + " is needed here and is not linked");
  return f;
}
int host_typed(void*, int chrnum, uint32_t x, uint32_t y, int type, int sign) {
  static const auto f = resolve_host(&IIT_exists_with_divno_typed_signed, "IIT_exists_with_divno_typed_signed");
  return f(g.iit, g.divint_crosstable[chrnum], x, y, type == GSNAPDP_DONOR ? g.donor_typeint : g.acceptor_typeint,
           sign) ? 1 : 0;
}
int host_low(void*, int chrnum, uint32_t x, int sign) {
  static const auto f = resolve_host(&IIT_low_exists_signed_p, "IIT_low_exists_signed_p");
  return f(g.iit, g.divint_crosstable[chrnum], x, sign) ? 1 : 0;
}
int host_high(void*, int chrnum, uint32_t x, int sign) {
  static const auto f = resolve_host(&IIT_high_exists_signed_p, "IIT_high_exists_signed_p");
  return f(g.iit, g.divint_crosstable[chrnum], x, sign) ? 1 : 0;
}
int host_exact(void*, int chrnum, uint32_t x, uint32_t y, int sign) {
  static const auto f = resolve_host(&IIT_exists_with_divno_signed, "IIT_exists_with_divno_signed");
  return f(g.iit, g.divint_crosstable[chrnum], x, y, sign) ? 1 : 0;
}
// The host's IIT as the batched ABI asks it: written by Dynprog_setup (before
// any aligner thread runs), only read by gmap's worker threads.
gsnapdp_iit g_host_iit;
void host_iit_setup() {
  gsnapdp_iit& x = g_host_iit;
  x.user = nullptr;
  x.site_level = g.donor_typeint >= 0 && g.acceptor_typeint >= 0 ? 1 : 0;
  x.pad = 0;
  x.typed = host_typed;
  x.low = host_low;
  x.high = host_high;
  x.exact = host_exact;
}
const gsnapdp_iit* host_iit() { return &g_host_iit; }

// Appends one window's known-site record (left_known[L2L], right_known[L2R],
// the KNOWN_INTRONS pair list) to `q` at `at` and returns its known_mode.
int known_site_record(std::vector<char>& q, size_t at, int chrnum, unsigned chrpos,
                      unsigned genomiclength, int leftoffset, int rightoffset, int L2L, int L2R,
                      int cdna_direction, bool watsonp) {
  // the two site arrays and room for a few known introns; a longer intron list
  // (KNOWN_INTRONS mode) asks again with the length the first call reported
  int cap = (int)std::min<size_t>((size_t)L2L + (size_t)L2R + 2 + 4 * 64, 0x7fffffff);
  int len = 0, mode = -1;
  for (int tries = 0; tries < 2 && mode < 0; tries++) {
    q.resize(at + (size_t)cap);
    mode = gsnapdp_known_site_record(host_iit(), g.novelsplicingp ? 1 : 0, chrnum, chrpos, genomiclength, leftoffset,
                                     rightoffset, L2L, L2R, cdna_direction, watsonp ? 1 : 0, q.data() + at, cap, &len);
    if (mode < 0 && len > cap) cap = len;
    else break;
  }
  if (mode < 0) fatal(std::string("known-site record: ") + gsnapdp_last_error());
  q.resize(at + (size_t)len + 8, 0);
  return mode;
}

SolveFn solver(bool end5) {
  SolveFn f = end5 ? &Splicetrie_solve_end5 : &Splicetrie_solve_end3;
  if (f) return f;
  f = (SolveFn)dlsym(RTLD_DEFAULT, end5 ? "Splicetrie_solve_end5" : "Splicetrie_solve_end3");
  if (!f) fatal("Splicetrie_solve_end5/3 not found: link the host program's splicetrie.o");
  return f;
}

}  // namespace

extern "C" {

static const int stats_order[6] = {F_GAP, F_SJ, F_GGAP, F_CGAP, F_MICRO, F_MAXENT};

// the round-1 layout, kept for existing callers: windows per family, then the
// gap family's batch count and largest batch
int Gsnapdp_dropin_stats(unsigned long* out, int n) {
  std::lock_guard<std::mutex> lock(gb.m);
  for (int i = 0; i < 6 && i < n; i++) out[i] = gb.windows[stats_order[i]];
  if (n > 6) out[6] = gb.batches[F_GAP];
  if (n > 7) out[7] = gb.maxbatch[F_GAP];
  return 8;
}

int Gsnapdp_dropin_stats2(unsigned long* out, int n) {
  std::lock_guard<std::mutex> lock(gb.m);
  for (int i = 0; i < 6; i++) {
    if (i < n) out[i] = gb.windows[stats_order[i]];
    if (6 + i < n) out[6 + i] = gb.batches[stats_order[i]];
    if (12 + i < n) out[12 + i] = gb.maxbatch[stats_order[i]];
  }
  return 18;
}

// every family, score_introns' k_introns launches included (7 x 3 values)
int Gsnapdp_dropin_stats3(unsigned long* out, int n) {
  static const int order[7] = {F_GAP, F_SJ, F_GGAP, F_CGAP, F_MICRO, F_MAXENT, F_INTRONS};
  std::lock_guard<std::mutex> lock(gb.m);
  for (int i = 0; i < 7; i++) {
    if (i < n) out[i] = gb.windows[order[i]];
    if (7 + i < n) out[7 + i] = gb.batches[order[i]];
    if (14 + i < n) out[14 + i] = gb.maxbatch[order[i]];
  }
  return 21;
}

int Gsnapdp_dropin_genome(const unsigned int* blocks, size_t nwords, int device) {
  std::lock_guard<std::mutex> lock(g.mu);
  if (g.ctx && (blocks != g.blocks || nwords != g.nwords)) fatal("genome changed after first use");
  g.blocks = blocks;
  g.nwords = nwords;
  g.device = device;
  g.explicit_genome = true;
  return 0;
}

char* Dynprog_endalign_string(gsnapdp_Endalign_T endalign) {  // dynprog.c:335-345
  switch (endalign) {
    case GSNAPDP_QUERYEND_GAP: return (char*)"queryend_gap";
    case GSNAPDP_QUERYEND_INDELS: return (char*)"queryend_indels";
    case GSNAPDP_QUERYEND_NOGAPS: return (char*)"queryend_nogaps";
    case GSNAPDP_BEST_LOCAL: return (char*)"best_local";
    default:
      printf("endalign %d not recognized\n", endalign);
      return (char*)"";
  }
}

// The splice sites and their tries feed Dynprog_end5/3_known; the splicing IIT
// feeds the known-site modes of bridge_intron_gap (Dynprog_genome_gap builds
// each window's known-site record from it with the host program's IIT calls).
void Dynprog_setup(gsnapdp_bool novelsplicingp, gsnapdp_IIT_T splicing_iit,
                   int* splicing_divint_crosstable, int donor_typeint, int acceptor_typeint,
                   gsnapdp_Genomicpos_T* splicesites, gsnapdp_Splicetype_T* splicetypes,
                   gsnapdp_Genomicpos_T*, int nsplicesites, unsigned int* trieoffsets_obs,
                   unsigned int* triecontents_obs, unsigned int* trieoffsets_max,
                   unsigned int* triecontents_max, gsnapdp_Genome_T genome) {
  std::lock_guard<std::mutex> lock(g.mu);
  if (genome && !g.explicit_genome && Genome_blocks && Genome_totallength) {
    unsigned int* blocks = Genome_blocks(genome);
    if (!blocks) fatal("Dynprog_setup: the genome is not in packed blocks (genomecomp)");
    if (g.ctx && blocks != g.blocks) fatal("genome changed after first use");
    g.blocks = blocks;
    g.nwords = (size_t)((Genome_totallength(genome) + 31U) / 32U) * 3;
  }
  g.splicing_iit = splicing_iit != nullptr;  // dynprog.c:358-366
  g.iit = splicing_iit;
  g.divint_crosstable = splicing_divint_crosstable;
  g.donor_typeint = donor_typeint;
  g.acceptor_typeint = acceptor_typeint;
  g.novelsplicingp = novelsplicingp != 0;
  g.splicesites = splicesites;
  g.splicetypes = splicetypes;
  g.nsplicesites = nsplicesites;
  g.trieoffsets_obs = trieoffsets_obs;
  g.triecontents_obs = triecontents_obs;
  g.trieoffsets_max = trieoffsets_max;
  g.triecontents_max = triecontents_max;
  host_iit_setup();
}

int Dynprog_score(int matches, int mismatches, int qopens, int qindels, int topens, int tindels,
                  double defect_rate) {  // dynprog.c:381-394 (open -10, extend -3 in every bin)
  const int mism = defect_rate < 0.003 ? -3 : (defect_rate < 0.014 ? -2 : -1);
  return 3 * matches + mism * mismatches - 10 * qopens - 3 * qindels - 10 * topens - 3 * tindels;
}

gsnapdp_Dynprog_T Dynprog_new(int maxlookback, int extraquerygap, int maxpeelback,
                              int extramaterial_end, int extramaterial_paired) {
  // compute_maxlengths, dynprog.c:831-852 (QUERY_MAXLENGTH 500, GENOMIC_MAXLENGTH 2000)
  int m1 = maxlookback + maxpeelback;
  if (m1 < 500) m1 = 500;
  int m2 = m1 + extraquerygap + (extramaterial_end > extramaterial_paired ? extramaterial_end
                                                                           : extramaterial_paired);
  if (m2 < 2000) m2 = 2000;
  Dynprog* d = new Dynprog{m1, m2};
  return (gsnapdp_Dynprog_T)d;
}

void Dynprog_free(gsnapdp_Dynprog_T* old) {
  if (old && *old) {
    delete (Dynprog*)*old;
    *old = nullptr;
  }
}

int Dynprog_pairdistance(int c1, int c2) {  // dynprog.c:1048 (HIGHQ table)
  return gsnapdp::host_pairdistance(0, c1, c2);
}

void Dynprog_term(void) {
  std::lock_guard<std::mutex> lock(g.mu);
  if (g.ctx) gsnapdp_destroy(g.ctx);
  g.ctx = nullptr;
  g.tables = false;
}

void Dynprog_init(int, int, int, int, int, gsnapdp_Mode_T mode) {  // dynprog.c:1339
  std::lock_guard<std::mutex> lock(g.mu);
  g.mode = mode;
  uint32_t prof[gsnapdp::PROF_WORDS];
  gsnapdp::build_profile_table(mode, prof);  // pairdistance_init for Dynprog_pairdistance
}

gsnapdp_List_T Dynprog_single_gap(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* sequence1, char* sequenceuc1, char*, char*,
    int length1, int length2, int offset1, int offset2, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_single,
    double defect_rate, int /*close_indels_mode: no effect, SURVEY A.14*/,
    gsnapdp_bool widebandp) {
  gsnapdp_window w = base_window(GSNAPDP_SINGLE_GAP, length1, length2, offset1, offset2,
                                 chroffset, chrhigh, chrpos, genomiclength, cdna_direction,
                                 watsonp, jump_late_p, extraband_single, defect_rate,
                                 (const Dynprog*)dynprog, *dynprogindex);
  w.widebandp = widebandp ? 1 : 0;
  return run_one(w, sequence1, sequenceuc1, false, pairpool, dynprogindex, finalscore, nmatches,
                 nmismatches, nopens, nindels);
}

gsnapdp_List_T Dynprog_end5_gap(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* revsequence1, char* revsequenceuc1, char*,
    char*, int length1, int length2, int revoffset1, int revoffset2,
    gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate, gsnapdp_Endalign_T endalign, gsnapdp_bool /*use_genomicseg_p*/) {
  gsnapdp_window w = base_window(GSNAPDP_END5_GAP, length1, length2, revoffset1, revoffset2,
                                 chroffset, chrhigh, chrpos, genomiclength, cdna_direction,
                                 watsonp, jump_late_p, extraband_end, defect_rate,
                                 (const Dynprog*)dynprog, *dynprogindex);
  w.widebandp = 1;
  w.endalign = (uint8_t)endalign;
  return run_one(w, revsequence1, revsequenceuc1, true, pairpool, dynprogindex, finalscore,
                 nmatches, nmismatches, nopens, nindels);
}

gsnapdp_List_T Dynprog_end3_gap(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* sequence1, char* sequenceuc1, char*, char*,
    int length1, int length2, int offset1, int offset2, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate, gsnapdp_Endalign_T endalign, gsnapdp_bool /*use_genomicseg_p*/) {
  gsnapdp_window w = base_window(GSNAPDP_END3_GAP, length1, length2, offset1, offset2, chroffset,
                                 chrhigh, chrpos, genomiclength, cdna_direction, watsonp,
                                 jump_late_p, extraband_end, defect_rate,
                                 (const Dynprog*)dynprog, *dynprogindex);
  w.widebandp = 1;
  w.endalign = (uint8_t)endalign;
  return run_one(w, sequence1, sequenceuc1, false, pairpool, dynprogindex, finalscore, nmatches,
                 nmismatches, nopens, nindels);
}

gsnapdp_List_T Dynprog_genome_gap(
    int* dynprogindex, int* finalscore, int* new_leftgenomepos, int* new_rightgenomepos,
    double* left_prob, double* right_prob, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, int* exonhead, int* introntype, gsnapdp_Dynprog_T dynprogL,
    gsnapdp_Dynprog_T dynprogR, char* sequence1, char* sequenceuc1, char*, char*, char*, char*,
    int length1, int length2L, int length2R, int offset1, int offset2L, int revoffset2R,
    int chrnum, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, char* /*genomicuc_ptr*/, gsnapdp_bool use_genomicseg_p,
    int cdna_direction, gsnapdp_bool watsonp, gsnapdp_bool jump_late_p,
    gsnapdp_Pairpool_T pairpool, int extraband_paired, double defect_rate, int maxpeelback,
    gsnapdp_bool halfp, gsnapdp_bool finalp, gsnapdp_bool use_probabilities_p,
    int score_threshold, gsnapdp_bool splicingp) {  // dynprog.c:4798-5061
  if (use_genomicseg_p && (use_probabilities_p || finalp))
    fatal("Dynprog_genome_gap: genomic-segment MaxEnt probabilities are not served");
  gsnapdp_ctx* c = shared_ctx(use_probabilities_p || finalp);
  const Dynprog* dL = (const Dynprog*)dynprogL;
  const Dynprog* dR = (const Dynprog*)dynprogR;
  GgapReq req;
  gsnapdp_ggap_window& w = req.w;
  memset(&w, 0, sizeof(w));
  w.length1 = length1;
  w.length2L = length2L;
  w.length2R = length2R;
  w.offset1 = offset1;
  w.offset2L = offset2L;
  w.revoffset2R = revoffset2R;
  w.chroffset = chroffset;
  w.chrhigh = chrhigh;
  w.chrpos = chrpos;
  w.genomiclength = genomiclength;
  w.qpos = 0;
  w.cdna_direction = cdna_direction;
  w.extraband_paired = extraband_paired;
  w.maxpeelback = maxpeelback;
  w.score_threshold = score_threshold;
  w.dynprogindex = *dynprogindex;
  // the two workspaces' limits (:4898-4927), folded into one exact test
  const bool too_long = length1 > dL->maxlength1 || length2L > dL->maxlength2 ||
                        length1 > dR->maxlength1 || length2R > dR->maxlength2;
  w.maxlength1 = too_long ? -1 : 0x3fffffff;
  w.maxlength2 = 0x3fffffff;
  w.defect_rate = defect_rate < 0.003 ? 0.001f : (defect_rate < 0.014 ? 0.01f : 0.5f);
  w.watsonp = watsonp ? 1 : 0;
  w.jump_late_p = jump_late_p ? 1 : 0;
  w.halfp = halfp ? 1 : 0;
  w.finalp = finalp ? 1 : 0;
  w.use_probabilities_p = use_probabilities_p ? 1 : 0;
  w.splicingp = splicingp ? 1 : 0;
  const int L1 = length1 > 0 ? length1 : 0;
  req.q.assign((size_t)L1 + 8, 0);
  req.qu.assign((size_t)L1 + 8, 0);
  if (L1 > 0) {
    memcpy(req.q.data(), sequence1, (size_t)L1);
    memcpy(req.qu.data(), sequenceuc1, (size_t)L1);
  }
  if (g.splicing_iit && L1 > 1 && length2L > 0 && length2R > 0 && !too_long) {
    // the known-site record follows the query rows (include/gsnapdp.h)
    w.known_mode = known_site_record(req.q, (size_t)L1, chrnum, chrpos, genomiclength,
                                     offset2L, revoffset2R, length2L, length2R, cdna_direction,
                                     watsonp != 0);
  }
  req.q.resize((req.q.size() + 3) & ~(size_t)3, 0);
  req.qu.resize(req.q.size(), 0);
  const int64_t cap = 2 * (int64_t)L1 + (length2L > 0 ? length2L : 0) + (length2R > 0 ? length2R : 0) + 4;
  req.cap = cap;
  submit(c, &req);
  const gsnapdp_ggap_result& r = req.r;
  const gsnapdp_ggap_trace& t = req.t;
  if (t.status == gsnapdp::ST_UNSUPPORTED)
    fatal("genome-gap window outside the reference's domain (the reference aborts or reads past its matrices)");
  if (t.status == gsnapdp::ST_OPS_OVERFLOW) fatal("op stream overflow");
  if (t.status == gsnapdp::ST_INTERNAL) fatal("genome-gap kernel invariant failed (bridge cell outside a flank)");
  // out-parameters exactly as the reference writes them on each path
  *nmatches = *nmismatches = *nopens = *nindels = 0;  // :4853-4854
  *left_prob = *right_prob = 0.0;
  *finalscore = r.finalscore;
  *dynprogindex = r.dynprogindex;
  if (t.status == gsnapdp::ST_EARLY) {
    if (too_long) {  // :4898-4927
      *new_leftgenomepos = r.new_leftgenomepos;
      *new_rightgenomepos = r.new_rightgenomepos;
      *exonhead = r.exonhead;
    }
    return nullptr;
  }
  // probability mode without a qualifying candidate reads uninitialised
  // indices in the reference (:4055); here it is defined as NULL, NEG_INFINITY
  if (r.bridge_ok == 0) return nullptr;
  // bridge_intron_gap writes *introntype only when a score-mode candidate is
  // taken (none taken leaves bestscore and bestscoreI at -100000), and always
  // in the constrained known-intron mode (NONINTRON, :3695)
  if (w.known_mode == GSNAPDP_KNOWN_INTRONS) *introntype = 0;
  else if (!use_probabilities_p && r.finalscore != (halfp ? -50000 : -100000)) *introntype = r.introntype;
  if (!t.bridge_accepted) return nullptr;  // bridge rejected (:4084-4101)
  *new_leftgenomepos = r.new_leftgenomepos;
  *new_rightgenomepos = r.new_rightgenomepos;
  *exonhead = r.exonhead;
  *left_prob = r.left_prob;
  *right_prob = r.right_prob;
  *nmatches = r.nmatches;
  *nmismatches = r.nmismatches;
  *nopens = r.nopens;
  *nindels = r.nindels;
  if (r.returned_null) return nullptr;  // only the gapholder (:5050-5053)
  thread_local std::vector<gsnapdp_pair> pairs;
  pairs.resize((size_t)cap + 8);
  const int n = gsnapdp_ggap_expand(c, &w, &r, &t, req.ops.data(), req.q.data(), req.qu.data(),
                                    pairs.data(), (int)pairs.size());
  if (n < 0 || n > (int)pairs.size()) fatal("gsnapdp_ggap_expand failed");
  return push_pairs(pairs.data(), n, pairpool);
}

gsnapdp_List_T Dynprog_cdna_gap(
    int* dynprogindex, int* finalscore, gsnapdp_bool* incompletep, gsnapdp_Dynprog_T dynprogL,
    gsnapdp_Dynprog_T dynprogR, char* sequence1L, char* sequenceuc1L, char* revsequence1R,
    char* revsequenceuc1R, char* sequence2, char* /*sequenceuc2*/, int length1L, int length1R,
    int length2, int offset1L, int revoffset1R, int offset2, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_paired,
    double defect_rate) {  // dynprog.c:4578-4793
  gsnapdp_ctx* c = shared_ctx(false);
  const Dynprog* dL = (const Dynprog*)dynprogL;
  const Dynprog* dR = (const Dynprog*)dynprogR;
  CgapReq req;
  gsnapdp_cgap_window& w = req.w;
  memset(&w, 0, sizeof(w));
  w.length1L = length1L;
  w.length1R = length1R;
  w.length2 = length2;
  w.offset1L = offset1L;
  w.revoffset1R = revoffset1R;
  w.offset2 = offset2;
  w.chroffset = chroffset;
  w.chrhigh = chrhigh;
  w.chrpos = chrpos;
  w.genomiclength = genomiclength;
  w.cdna_direction = cdna_direction;
  w.extraband_paired = extraband_paired;
  w.dynprogindex = *dynprogindex;
  // the two workspaces' limits (:4651-4675), folded into one exact test
  const bool too_long = length2 > dR->maxlength1 || length1R > dR->maxlength2 ||
                        length2 > dL->maxlength1 || length1L > dL->maxlength2;
  w.maxlength1 = too_long ? -1 : 0x3fffffff;
  w.maxlength2 = 0x3fffffff;
  w.defect_rate = defect_rate < 0.003 ? 0.001f : (defect_rate < 0.014 ? 0.01f : 0.5f);
  w.watsonp = watsonp ? 1 : 0;
  w.jump_late_p = jump_late_p ? 1 : 0;
  // the query the fills read: sequence1L[0 .. length1L) forwards and
  // revsequence1R[-(length1R-1) .. 0]; INSERT_PAIRS also reads sequence1L up to
  // revoffset1R - offset1L
  const int nL = length1L > 0 ? length1L : 0, nR = length1R > 0 ? length1R : 0;
  const int span = revoffset1R - offset1L + 1 > nL ? revoffset1R - offset1L + 1 : nL;
  req.q.assign(((size_t)span + nR + 8 + 3) & ~(size_t)3, 0);
  req.qu.assign(req.q.size(), 0);
  if (length2 > 1) {
    memcpy(req.q.data(), sequence1L, (size_t)span);
    memcpy(req.qu.data(), sequenceuc1L, (size_t)span);
    memcpy(req.q.data() + span, revsequence1R - (nR - 1), (size_t)nR);
    memcpy(req.qu.data() + span, revsequenceuc1R - (nR - 1), (size_t)nR);
  }
  w.qposL = 0;
  w.qposR = (uint32_t)(span + nR - 1);
  const int64_t cap = (int64_t)nL + nR + 2 * (int64_t)(length2 > 0 ? length2 : 0) + 4;
  req.cap = cap;
  submit(c, &req);
  const gsnapdp_cgap_result& r = req.r;
  if (r.status == gsnapdp::ST_UNSUPPORTED)
    fatal("cDNA-gap window outside the reference's domain (the reference aborts here)");
  if (r.status == gsnapdp::ST_OPS_OVERFLOW) fatal("op stream overflow");
  *dynprogindex = r.dynprogindex;
  if (r.finalscore_set) *finalscore = r.finalscore;
  // no bridge candidate: the reference traces back from uninitialised indices;
  // defined here as NULL with the bridge's score
  if (r.status != gsnapdp::ST_OK) return nullptr;
  if (r.incompletep) *incompletep = 1;  // only ever set to true (:4756)
  if (r.returned_null) return nullptr;
  thread_local std::vector<gsnapdp_pair> pairs;
  pairs.resize((size_t)cap + 32);
  const int n = gsnapdp_cgap_expand(c, &w, &r, req.ops.data(), req.q.data(), req.qu.data(), sequence2,
                                    pairs.data(), (int)pairs.size());
  if (n < 0 || n > (int)pairs.size()) fatal("gsnapdp_cgap_expand failed");
  return push_pairs(pairs.data(), n, pairpool);
}

gsnapdp_List_T Dynprog_end5_splicejunction(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* revsequence1, char* revsequenceuc1,
    char* revsequence2, char* revsequenceuc2, int length1, int length2, int revoffset1,
    int revoffset2_anchor, int revoffset2_far, gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T,
    gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate, int contlength) {
  return run_sj(GSNAPDP_END5_GAP, revsequence1, revsequenceuc1, revsequence2, revsequenceuc2,
                length1, length2, revoffset1, revoffset2_anchor, revoffset2_far, contlength,
                cdna_direction, watsonp, jump_late_p, extraband_end, defect_rate,
                (const Dynprog*)dynprog, pairpool, dynprogindex, finalscore, nmatches,
                nmismatches, nopens, nindels);
}

gsnapdp_List_T Dynprog_end3_splicejunction(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* sequence1, char* sequenceuc1,
    char* sequence2, char* sequenceuc2, int length1, int length2, int offset1,
    int offset2_anchor, int offset2_far, gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T,
    gsnapdp_Genomicpos_T, gsnapdp_Genomicpos_T, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate, int contlength) {
  return run_sj(GSNAPDP_END3_GAP, sequence1, sequenceuc1, sequence2, sequenceuc2, length1,
                length2, offset1, offset2_anchor, offset2_far, contlength, cdna_direction,
                watsonp, jump_late_p, extraband_end, defect_rate, (const Dynprog*)dynprog,
                pairpool, dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels);
}

void Dynprog_make_splicejunction_5(char* splicejunction, gsnapdp_Genomicpos_T splicecoord,
                                   int splicelength, int /*contlength*/,
                                   gsnapdp_Splicetype_T far_splicetype, gsnapdp_bool watsonp) {
  // dynprog.c:6061-6100: the distal part at splicejunction[0]
  char* distal = splicejunction;
  if (far_splicetype == ACCEPTOR || far_splicetype == ANTIDONOR) {
    if (splicelength > 0) fill_buffer(splicecoord, (unsigned)splicelength, distal);
  } else if (far_splicetype == ANTIACCEPTOR || far_splicetype == DONOR) {
    if (splicelength > 0) fill_buffer(splicecoord - (unsigned)splicelength, (unsigned)splicelength, distal);
  } else {
    fprintf(stderr, "Unexpected far_splicetype value %d\n", far_splicetype);
    abort();
  }
  if (!watsonp) revcomp_inplace(distal, splicelength);
}

void Dynprog_make_splicejunction_3(char* splicejunction, gsnapdp_Genomicpos_T splicecoord,
                                   int splicelength, int contlength,
                                   gsnapdp_Splicetype_T far_splicetype, gsnapdp_bool watsonp) {
  // dynprog.c:6149-6188: the distal part after the contlength proximal bases
  char* distal = &splicejunction[contlength];
  if (far_splicetype == DONOR || far_splicetype == ANTIACCEPTOR) {
    if (splicelength > 0) fill_buffer(splicecoord - (unsigned)splicelength, (unsigned)splicelength, distal);
  } else if (far_splicetype == ANTIDONOR || far_splicetype == ACCEPTOR) {
    if (splicelength > 0) fill_buffer(splicecoord, (unsigned)splicelength, distal);
  } else {
    fprintf(stderr, "Unexpected far_splicetype value %d\n", far_splicetype);
    abort();
  }
  if (!watsonp) revcomp_inplace(distal, splicelength);
}

gsnapdp_List_T Dynprog_microexon_int(
    double* bestprob2, double* bestprob3, int* dynprogindex, int* microintrontype,
    char* sequence1, char* sequenceuc1, char*, char*, char*, char*, int length1, int, int,
    int offset1, int offset2L, int revoffset2R, int cdna_direction, char* queryseq,
    char* queryuc, char*, char*, gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
    gsnapdp_Genomicpos_T chrpos, gsnapdp_Genomicpos_T genomiclength, gsnapdp_bool watsonp,
    gsnapdp_bool use_genomicseg_p, gsnapdp_Pairpool_T pairpool, double defect_rate) {
  *bestprob2 = *bestprob3 = 0.0;  // :7168
  if (cdna_direction == 0) {      // :7203-7206
    fprintf(stderr, "cdna_direction is 0 in Dynprog_microexon_int\n");
    abort();
  }
  if (revoffset2R - offset2L <= 0) {  // :7222-7225
    fprintf(stderr, "Bug in Dynprog_microexon_int.  span %d <= 0.  Please report to twu@gene.com\n",
            revoffset2R - offset2L);
    abort();
  }
  if (use_genomicseg_p) fatal("Dynprog_microexon_int with use_genomicseg_p (no caller passes it)");
  gsnapdp_ctx* c = shared_ctx(true);
  MicroReq req;
  const int L1 = length1 > 0 ? length1 : 0;
  // sequence1 / sequenceuc1 for the search, queryseq / queryuc from offset1 for the pairs
  const size_t pbase = ((size_t)L1 + 8 + 3) & ~(size_t)3;
  req.q.assign(pbase + (((size_t)L1 + 8 + 3) & ~(size_t)3), 0);
  req.qu.assign(req.q.size(), 0);
  if (L1 > 0) {
    memcpy(req.q.data(), sequence1, (size_t)L1);
    memcpy(req.qu.data(), sequenceuc1, (size_t)L1);
    memcpy(req.q.data() + pbase, queryseq + offset1, (size_t)L1);
    memcpy(req.qu.data() + pbase, queryuc + offset1, (size_t)L1);
  }
  gsnapdp_micro_window& w = req.w;
  memset(&w, 0, sizeof(w));
  w.length1 = length1;
  w.offset1 = offset1;
  w.offset2L = offset2L;
  w.revoffset2R = revoffset2R;
  w.cdna_direction = cdna_direction;
  w.dynprogindex = *dynprogindex;
  w.chroffset = chroffset;
  w.chrhigh = chrhigh;
  w.chrpos = chrpos;
  w.genomiclength = genomiclength;
  w.qpos = 0;
  w.ppos = (uint32_t)pbase;
  w.defect_rate = defect_rate < 0.003 ? 0.001f : (defect_rate < 0.014 ? 0.01f : 0.5f);
  w.watsonp = watsonp ? 1 : 0;
  submit(c, &req);
  const gsnapdp_micro_result& r = req.r;
  if (r.status != 0) fatal("microexon window outside the reference's domain");
  *bestprob2 = r.bestprob2;
  *bestprob3 = r.bestprob3;
  *microintrontype = r.microintrontype;
  *dynprogindex = r.dynprogindex;
  if (!r.found) return nullptr;
  thread_local std::vector<gsnapdp_pair> pairs;
  pairs.resize((size_t)L1 + 4);
  const int n = gsnapdp_micro_expand(c, &w, &r, req.q.data(), req.qu.data(), pairs.data(),
                                     (int)pairs.size());
  if (n <= 0 || n > (int)pairs.size()) fatal("gsnapdp_micro_expand failed");
  gsnapdp_List_T list = nullptr;
  for (int i = n - 1; i >= 0; i--) {
    const gsnapdp_pair& p = pairs[(size_t)i];
    if (p.gapp) {
      list = Pairpool_push_gapholder(list, pairpool, p.queryjump, p.genomejump, 0);
      ((RefPairHead*)((RefList*)list)->first)->comp = p.comp;  // gappair->comp = gapchar
    } else {
      list = Pairpool_push(list, pairpool, p.querypos, p.genomepos, p.cdna, p.comp, p.genome,
                           p.dynprogindex);
    }
  }
  return list;
}

// Dynprog_end5_known (dynprog.c:6414-6677): the plain QUERYEND_NOGAPS end gap,
// then every anchor splice site of the right type in the end's genomic range
// tried through the host program's Splicetrie_solve_end5 (which calls back
// into Dynprog_make_splicejunction_5 / Dynprog_end5_splicejunction here), then
// the reference's fallbacks: BEST_LOCAL when nothing spliced, or the ambiguous
// part cut off.  Host control flow; every DP runs on the GPU.
gsnapdp_List_T Dynprog_end5_known(
    gsnapdp_bool* knownsplicep, int* dynprogindex, int* finalscore, int* ambig_end_length,
    gsnapdp_Splicetype_T* ambig_splicetype, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* revsequence1, char* revsequenceuc1,
    char* revsequence2, char* revsequenceuc2, int length1, int length2, int revoffset1,
    int revoffset2, gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
    gsnapdp_Genomicpos_T chrpos, int genomiclength, gsnapdp_Genomicpos_T knownsplice_limit_low,
    gsnapdp_Genomicpos_T knownsplice_limit_high, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate) {
  const Dynprog* dp = (const Dynprog*)dynprog;
  *ambig_end_length = 0;
  if (length1 <= 0 || length2 <= 0) {  // :6451-6464
    *finalscore = 0;
    *knownsplicep = 0;
    return nullptr;
  }
  const int perfect_score = length1 * 3;
  const SolveFn solve = solver(true);
  gsnapdp_List_T best_pairs = Dynprog_end5_gap(
      dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dynprog, revsequence1,
      revsequenceuc1, revsequence2, revsequenceuc2, length1, length2, revoffset1, revoffset2,
      chroffset, chrhigh, chrpos, (gsnapdp_Genomicpos_T)genomiclength, cdna_direction, watsonp,
      jump_late_p, pairpool, extraband_end, defect_rate, GSNAPDP_QUERYEND_NOGAPS, 0);
  const int orig_score = *finalscore;
  gsnapdp_List_T orig_pairs = best_pairs;
  int threshold_miss_score = perfect_score - orig_score;
  *knownsplicep = 0;
  int anchor_splicetype = 0;
  if (threshold_miss_score > 0 && length2 > 0) {  // :6488-6602
    std::vector<char> splicejunction((size_t)length2 + 1, 0);
    const int endlength = length1;
    unsigned low, high;
    int far_splicetype;
    if (watsonp) {
      low = chroffset + chrpos + (unsigned)(revoffset2 - endlength + 2);
      high = chroffset + chrpos + (unsigned)(revoffset2 + 1);
      anchor_splicetype = cdna_direction > 0 ? ACCEPTOR : ANTIDONOR;
      far_splicetype = cdna_direction > 0 ? DONOR : ANTIACCEPTOR;
    } else {
      low = chroffset + chrpos + (unsigned)(genomiclength - 1) - (unsigned)revoffset2;
      high = chroffset + chrpos + (unsigned)(genomiclength - 1) - (unsigned)(revoffset2 - endlength) - 1u;
      anchor_splicetype = cdna_direction > 0 ? ANTIACCEPTOR : DONOR;
      far_splicetype = cdna_direction > 0 ? ANTIDONOR : ACCEPTOR;
    }
    unsigned far_limit_low = knownsplice_limit_low, far_limit_high = knownsplice_limit_high;
    int j = binary_search(0, g.nsplicesites, g.splicesites, low);
    while (j < g.nsplicesites && g.splicesites[j] <= high) {
      if (g.splicetypes[j] == anchor_splicetype) {
        const int contlength = watsonp ? (int)(high - g.splicesites[j]) : (int)(g.splicesites[j] - low);
        const int splicelength = length2 - contlength;
        // make_contjunction_5 (dynprog.c:5998-6035): the proximal part after the distal one
        char* proximal = &splicejunction[(size_t)splicelength];
        if (anchor_splicetype == ACCEPTOR || anchor_splicetype == ANTIDONOR)
          fill_buffer(g.splicesites[j], (unsigned)contlength, proximal);
        else
          fill_buffer(g.splicesites[j] - (unsigned)contlength, (unsigned)contlength, proximal);
        if (!watsonp) revcomp_inplace(proximal, contlength);
        if (watsonp) far_limit_high = g.splicesites[j];
        else far_limit_low = g.splicesites[j];
        int obsmax_penalty = 0;
        if (g.trieoffsets_obs != nullptr) {
          best_pairs = solve(
              best_pairs, g.triecontents_obs, g.trieoffsets_obs, j, far_limit_low, far_limit_high,
              finalscore, nmatches, nmismatches, nopens, nindels, knownsplicep, ambig_end_length,
              &threshold_miss_score, 0, perfect_score, g.splicesites[j], splicejunction.data(),
              splicelength, contlength, far_splicetype, chroffset, chrhigh, chrpos, genomiclength,
              dynprogindex, dynprog, revsequence1, revsequenceuc1, length1, length2, revoffset1,
              revoffset2, cdna_direction, watsonp, jump_late_p, pairpool, extraband_end,
              defect_rate);
          obsmax_penalty += 3;  // FULLMATCH
        }
        if (threshold_miss_score - obsmax_penalty > 0 && g.trieoffsets_max != nullptr) {
          best_pairs = solve(
              best_pairs, g.triecontents_max, g.trieoffsets_max, j, far_limit_low, far_limit_high,
              finalscore, nmatches, nmismatches, nopens, nindels, knownsplicep, ambig_end_length,
              &threshold_miss_score, obsmax_penalty, perfect_score, g.splicesites[j],
              splicejunction.data(), splicelength, contlength, far_splicetype, chroffset, chrhigh,
              chrpos, genomiclength, dynprogindex, dynprog, revsequence1, revsequenceuc1, length1,
              length2, revoffset1, revoffset2, cdna_direction, watsonp, jump_late_p, pairpool,
              extraband_end, defect_rate);
        }
      }
      j++;
    }
  }
  if (best_pairs == nullptr) {  // :6605-6660
    if (*ambig_end_length == 0) {
      if (length1 > dp->maxlength1) length1 = dp->maxlength1;
      if (length2 > dp->maxlength2) length2 = dp->maxlength2;
      orig_pairs = Dynprog_end5_gap(
          dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dynprog,
          revsequence1, revsequenceuc1, revsequence2, revsequenceuc2, length1, length2,
          revoffset1, revoffset2, chroffset, chrhigh, chrpos, (gsnapdp_Genomicpos_T)genomiclength,
          cdna_direction, watsonp, jump_late_p, pairpool, extraband_end, defect_rate,
          GSNAPDP_BEST_LOCAL, 0);
      *knownsplicep = 0;
      return orig_pairs;
    }
    *ambig_splicetype = anchor_splicetype;
    orig_pairs = List_reverse(orig_pairs);  // truncate the ambiguous part; querypos increasing
    while (orig_pairs != nullptr &&
           ((RefPairHead*)((RefList*)orig_pairs)->first)->querypos < *ambig_end_length) {
      void* pair;
      orig_pairs = Pairpool_pop(orig_pairs, &pair);
    }
    orig_pairs = List_reverse(orig_pairs);
    *knownsplicep = 0;
    *finalscore = orig_score;
    return orig_pairs;
  }
  *ambig_end_length = 0;
  return *knownsplicep ? Pair_protect(best_pairs) : best_pairs;
}

// Dynprog_end3_known (dynprog.c:6680-6943), the 3' mirror of the above.
gsnapdp_List_T Dynprog_end3_known(
    gsnapdp_bool* knownsplicep, int* dynprogindex, int* finalscore, int* ambig_end_length,
    gsnapdp_Splicetype_T* ambig_splicetype, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* sequence1, char* sequenceuc1,
    char* sequence2, char* sequenceuc2, int length1, int length2, int offset1, int offset2,
    int querylength, gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
    gsnapdp_Genomicpos_T chrpos, int genomiclength, gsnapdp_Genomicpos_T knownsplice_limit_low,
    gsnapdp_Genomicpos_T knownsplice_limit_high, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate) {
  const Dynprog* dp = (const Dynprog*)dynprog;
  *ambig_end_length = 0;
  if (length1 <= 0 || length2 <= 0) {  // :6716-6729
    *finalscore = 0;
    *knownsplicep = 0;
    return nullptr;
  }
  const int perfect_score = length1 * 3;
  const SolveFn solve = solver(false);
  gsnapdp_List_T best_pairs = Dynprog_end3_gap(
      dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dynprog, sequence1,
      sequenceuc1, sequence2, sequenceuc2, length1, length2, offset1, offset2, chroffset,
      chrhigh, chrpos, (gsnapdp_Genomicpos_T)genomiclength, cdna_direction, watsonp, jump_late_p,
      pairpool, extraband_end, defect_rate, GSNAPDP_QUERYEND_NOGAPS, 0);
  const int orig_score = *finalscore;
  gsnapdp_List_T orig_pairs = best_pairs;
  int threshold_miss_score = perfect_score - orig_score;
  *knownsplicep = 0;
  int anchor_splicetype = 0;
  if (threshold_miss_score > 0 && length2 > 0) {  // :6753-6866
    std::vector<char> splicejunction((size_t)length2 + 1, 0);
    const int endlength = length1;
    unsigned low, high;
    int far_splicetype;
    if (watsonp) {
      low = chroffset + chrpos + (unsigned)offset2;
      high = chroffset + chrpos + (unsigned)(offset2 + endlength - 1);
      anchor_splicetype = cdna_direction > 0 ? DONOR : ANTIACCEPTOR;
      far_splicetype = cdna_direction > 0 ? ACCEPTOR : ANTIDONOR;
    } else {
      low = chroffset + chrpos + (unsigned)(genomiclength - 1) - (unsigned)(offset2 + endlength) + 2u;
      high = chroffset + chrpos + (unsigned)(genomiclength - 1) - (unsigned)offset2 + 1u;
      anchor_splicetype = cdna_direction > 0 ? ANTIDONOR : ACCEPTOR;
      far_splicetype = cdna_direction > 0 ? ANTIACCEPTOR : DONOR;
    }
    unsigned far_limit_low = knownsplice_limit_low, far_limit_high = knownsplice_limit_high;
    int j = binary_search(0, g.nsplicesites, g.splicesites, low);
    while (j < g.nsplicesites && g.splicesites[j] <= high) {
      if (g.splicetypes[j] == anchor_splicetype) {
        const int contlength = watsonp ? (int)(g.splicesites[j] - low) : (int)(high - g.splicesites[j]);
        const int splicelength = length2 - contlength;
        // make_contjunction_3 (dynprog.c:6103-6140): the proximal part first
        char* proximal = splicejunction.data();
        if (anchor_splicetype == DONOR || anchor_splicetype == ANTIACCEPTOR)
          fill_buffer(g.splicesites[j] - (unsigned)contlength, (unsigned)contlength, proximal);
        else
          fill_buffer(g.splicesites[j], (unsigned)contlength, proximal);
        if (!watsonp) revcomp_inplace(proximal, contlength);
        if (watsonp) far_limit_low = g.splicesites[j];
        else far_limit_high = g.splicesites[j];
        int obsmax_penalty = 0;
        if (g.trieoffsets_obs != nullptr) {
          best_pairs = solve(
              best_pairs, g.triecontents_obs, g.trieoffsets_obs, j, far_limit_low, far_limit_high,
              finalscore, nmatches, nmismatches, nopens, nindels, knownsplicep, ambig_end_length,
              &threshold_miss_score, 0, perfect_score, g.splicesites[j], splicejunction.data(),
              splicelength, contlength, far_splicetype, chroffset, chrhigh, chrpos, genomiclength,
              dynprogindex, dynprog, sequence1, sequenceuc1, length1, length2, offset1, offset2,
              cdna_direction, watsonp, jump_late_p, pairpool, extraband_end, defect_rate);
          obsmax_penalty += 3;  // FULLMATCH
        }
        if (threshold_miss_score - obsmax_penalty > 0 && g.trieoffsets_max != nullptr) {
          best_pairs = solve(
              best_pairs, g.triecontents_max, g.trieoffsets_max, j, far_limit_low, far_limit_high,
              finalscore, nmatches, nmismatches, nopens, nindels, knownsplicep, ambig_end_length,
              &threshold_miss_score, obsmax_penalty, perfect_score, g.splicesites[j],
              splicejunction.data(), splicelength, contlength, far_splicetype, chroffset, chrhigh,
              chrpos, genomiclength, dynprogindex, dynprog, sequence1, sequenceuc1, length1,
              length2, offset1, offset2, cdna_direction, watsonp, jump_late_p, pairpool,
              extraband_end, defect_rate);
        }
      }
      j++;
    }
  }
  if (best_pairs == nullptr) {  // :6869-6930
    if (*ambig_end_length == 0) {
      if (length1 > dp->maxlength1) length1 = dp->maxlength1;
      if (length2 > dp->maxlength2) length2 = dp->maxlength2;
      orig_pairs = Dynprog_end3_gap(
          dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dynprog, sequence1,
          sequenceuc1, sequence2, sequenceuc2, length1, length2, offset1, offset2, chroffset,
          chrhigh, chrpos, (gsnapdp_Genomicpos_T)genomiclength, cdna_direction, watsonp,
          jump_late_p, pairpool, extraband_end, defect_rate, GSNAPDP_BEST_LOCAL, 0);
      *knownsplicep = 0;
      return orig_pairs;
    }
    *ambig_splicetype = anchor_splicetype;
    // truncate the ambiguous part; querypos decreasing
    while (orig_pairs != nullptr && ((RefPairHead*)((RefList*)orig_pairs)->first)->querypos >=
                                        querylength - *ambig_end_length) {
      void* pair;
      orig_pairs = Pairpool_pop(orig_pairs, &pair);
    }
    *knownsplicep = 0;
    *finalscore = orig_score;
    return orig_pairs;
  }
  *ambig_end_length = 0;
  return *knownsplicep ? Pair_protect(best_pairs) : best_pairs;
}

void Maxent_hr_setup(unsigned int* ref_blocks) {  // maxent_hr.c:27195
  std::lock_guard<std::mutex> lock(g.mu);
  if (g.blocks && ref_blocks != g.blocks) fatal("Maxent_hr_setup blocks differ from the genome");
  if (!g.blocks) g.blocks = ref_blocks;  // sized in ctx() unless Dynprog_setup sizes it
}

// score_introns (stage3.c:7935-8162), the reference's static function with its
// signature (non-WASTE build), for a stage3.c that calls it here: the path's
// introns are picked on the host (gsnapdp_path_introns), the splicing IIT of
// Dynprog_setup (= Stage3_setup's, gmap.c:3828-3835) is asked about each site
// exactly where the reference asks, and the MaxEnt probabilities, sums and
// averages run in one k_introns launch shared with concurrent callers.  The
// returned list is the path's own cells in reverse order, which is what the
// reference's pop / List_push_existing loop builds.
gsnapdp_List_T Gsnapdp_score_introns(double* avg_donor_score, double* avg_acceptor_score, int* nbadintrons,
                                     gsnapdp_List_T path, int cdna_direction, gsnapdp_bool watsonp, int chrnum,
                                     gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
                                     gsnapdp_Genomicpos_T chrpos, char* genomicuc_ptr, int genomiclength,
                                     int nullgap, gsnapdp_bool use_genomicseg_p) {
  (void)chrhigh;
  (void)genomicuc_ptr;
  if (use_genomicseg_p) fatal("score_introns on a genomic segment (maxent.c) is not served");
  std::vector<gsnapdp_path_pair> pp;
  for (const RefList* l = (const RefList*)path; l; l = l->rest) {
    const RefPairGap* x = (const RefPairGap*)l->first;
    gsnapdp_path_pair q;
    q.genomepos = x->genomepos;
    q.queryjump = x->queryjump;
    q.genomejump = x->genomejump;
    q.gapp = x->gapp;
    q.knowngapp = x->knowngapp;
    q.comp = (uint8_t)x->comp;
    q.pad = 0;
    pp.push_back(q);
  }
  IntronReq req;
  const int n = gsnapdp_path_introns(pp.data(), (int)pp.size(), nullgap, 0, nullptr, 0);
  if (n < 0) fatal("score_introns: an intron at the end of the path (the reference dereferences NULL)");
  req.introns.resize((size_t)n);
  gsnapdp_path_introns(pp.data(), (int)pp.size(), nullgap, 0, req.introns.data(), n);
  if (g.iit && gsnapdp_introns_known(host_iit(), chrnum, chrpos, genomiclength, cdna_direction, watsonp ? 1 : 0,
                                     req.introns.data(), n))  // known sites score 1.0 (:7997-8046, :8069-8116)
    fatal(std::string("score_introns: ") + gsnapdp_last_error());
  req.p.chroffset = chroffset;
  req.p.chrpos = chrpos;
  req.p.genomiclength = genomiclength;
  req.p.cdna_direction = cdna_direction;
  req.p.watsonp = watsonp ? 1 : 0;
  req.p.first_intron = 0;
  req.p.nintrons = n;
  req.p.pad = 0;
  submit(shared_ctx(true), &req);
  *avg_donor_score = req.out.avg_donor_score;
  *avg_acceptor_score = req.out.avg_acceptor_score;
  *nbadintrons = req.out.nbadintrons;
  return path ? List_reverse(path) : path;
}

}  // extern "C"

namespace {

// ---- traverse_dual_break's stage 2, served by the host program (the pass's
// stage-2 callback).  Each Gsnapdp_build_dual_breaks call registers its
// Stage2_compute_one arguments under a tag the pass hands back (`invocation`).
struct Stage2Args {
  char *queryseq_ptr, *queryuc_ptr, *genomicseg_ptr, *genomicuc_ptr;
  int genestrand, watsonp;
  void* oligoindices;
  int noligoindices;
  gsnapdp_Pairpool_T pairpool;
  void* diagpool;
  int sufflookback, nsufflookback, maxintronlen;
};
std::mutex g_s2_mu;
std::unordered_map<int, Stage2Args*> g_s2_calls;
int g_s2_next = 0;
int stage2_register(Stage2Args* a) {
  std::lock_guard<std::mutex> l(g_s2_mu);
  const int id = g_s2_next++ & 0x3fffffff;
  g_s2_calls[id] = a;
  return id;
}
void stage2_unregister(int id) {
  std::lock_guard<std::mutex> l(g_s2_mu);
  g_s2_calls.erase(id);
}
int host_stage2(void*, const gsnapdp_s3_call* c, int querydp5, int querydp3, int, int, uint32_t mappingstart,
                uint32_t mappingend, gsnapdp_s3_pair* out, int cap) {
  Stage2Args* a;
  {
    std::lock_guard<std::mutex> l(g_s2_mu);
    auto it = g_s2_calls.find(c->invocation);
    if (it == g_s2_calls.end()) return -1;
    a = it->second;
  }
  static const auto f = resolve_host(&Stage2_compute_one, "Stage2_compute_one");
  const uint32_t genomicstart = c->chroffset + c->chrpos, genomicend = genomicstart + (uint32_t)c->genomiclength;
  int source = 0, indexsize = 0;
  // :7104-7117, as traverse_dual_break calls it
  gsnapdp_List_T l = f(&source, &indexsize, a->queryseq_ptr + querydp5, a->queryuc_ptr + querydp5,
                       querydp3 - querydp5 + 1, querydp5, a->genomicseg_ptr, a->genomicuc_ptr, genomicstart,
                       genomicend, mappingstart, mappingend, a->watsonp, a->genestrand, c->genomiclength,
                       a->oligoindices, a->noligoindices, 0.80, a->pairpool, a->diagpool, a->sufflookback,
                       a->nsufflookback, a->maxintronlen, /*localp*/ 1, /*skip_repetitive_p*/ 0,
                       /*use_shifted_canonical_p*/ 1, /*favor_right_p*/ 0, 0, 0, nullptr, 0);
  int n = 0;
  for (const RefList* p = (const RefList*)l; p; p = p->rest, n++) {
    if (n >= cap) continue;
    const RefPair* x = (const RefPair*)p->first;
    gsnapdp_s3_pair& o = out[n];
    o.querypos = x->querypos;
    o.genomepos = (int32_t)x->genomepos;
    o.queryjump = x->queryjump;
    o.genomejump = x->genomejump;
    o.dynprogindex = x->dynprogindex;
    o.src = -1;
    o.cdna = x->cdna;
    o.comp = x->comp;
    o.genome = x->genome;
    o.flags = (uint8_t)((x->gapp ? GSNAPDP_S3_GAPP : 0) | (x->knowngapp ? GSNAPDP_S3_KNOWNGAPP : 0) |
                        (x->disallowedp ? GSNAPDP_S3_DISALLOWED : 0) | (x->shortexonp ? GSNAPDP_S3_SHORTEXON : 0) |
                        (x->end_intron_p ? GSNAPDP_S3_END_INTRON : 0));
  }
  return n;
}

// One path through gsnapdp_stage3_pass_compact (k holds the call's arguments and
// in-counters) and back as the reference's list: its own cells for the pairs it
// keeps (disallowedp set where the reference sets it, stage3.c:5873-5880) and the
// host's Pairpool for the pairs the fills made.
gsnapdp_List_T pass_one(gsnapdp_s3_call& k, gsnapdp_List_T path, char* queryseq_ptr, char* queryuc_ptr,
                        gsnapdp_Pairpool_T pairpool, const gsnapdp_iit* iit, const char* what) {
  gsnapdp_ctx* c = shared_ctx(true);
  if (k.pass == GSNAPDP_S3_DUALBREAKS) {  // the host's stage 2 for traverse_dual_break (a context may be new)
    const gsnapdp_s3_stage2 s2 = {nullptr, host_stage2};
    gsnapdp_stage3_set_stage2(c, &s2);
  }
  thread_local std::vector<RefList*> incells;  // per gmap worker thread
  thread_local std::vector<gsnapdp_s3_pair> in;
  incells.clear();
  in.clear();
  for (RefList* l = (RefList*)path; l; l = l->rest) {
    const RefPair* x = (const RefPair*)l->first;
    gsnapdp_s3_pair p;
    p.querypos = x->querypos;
    p.genomepos = (int32_t)x->genomepos;
    p.queryjump = x->queryjump;
    p.genomejump = x->genomejump;
    p.dynprogindex = x->dynprogindex;
    p.src = (int32_t)incells.size();
    p.cdna = x->cdna;
    p.comp = x->comp;
    p.genome = x->genome;
    p.flags = (uint8_t)((x->gapp ? GSNAPDP_S3_GAPP : 0) | (x->knowngapp ? GSNAPDP_S3_KNOWNGAPP : 0) |
                        (x->disallowedp ? GSNAPDP_S3_DISALLOWED : 0) | (x->shortexonp ? GSNAPDP_S3_SHORTEXON : 0) |
                        (x->end_intron_p ? GSNAPDP_S3_END_INTRON : 0));
    in.push_back(p);
    incells.push_back(l);
  }
  k.npairs = (int32_t)in.size();
  const int64_t cap = 2 * ((int64_t)k.querylength + k.npairs) + 64;
  thread_local std::vector<int32_t> cells;  // the returned list, compactly
  thread_local std::vector<gsnapdp_s3_pair> news;
  cells.resize((size_t)cap);
  news.resize((size_t)cap);  // every new pair is one returned cell
  gsnapdp_s3_stats st;
  const gsnapdp_s3_call k0 = k;
  int rc = gsnapdp_stage3_pass_compact(c, &k, 1, in.data(), (int64_t)in.size(), queryseq_ptr, queryuc_ptr,
                                       (size_t)k.querylength, iit, cells.data(), cap, news.data(),
                                       (int64_t)news.size(), &st);
  if (rc && st.new_pairs > (int64_t)news.size()) {  // the pass reported what it needs: once more with room
    k = k0;
    news.resize((size_t)st.new_pairs);
    rc = gsnapdp_stage3_pass_compact(c, &k, 1, in.data(), (int64_t)in.size(), queryseq_ptr, queryuc_ptr,
                                     (size_t)k.querylength, iit, cells.data(), cap, news.data(),
                                     (int64_t)news.size(), &st);
  }
  if (rc) fatal(std::string("gsnapdp_stage3_pass_compact: ") + gsnapdp_last_error());
  if (k.status) fatal(std::string(what) + ": a window outside the reference's domain (the reference aborts)");
  gsnapdp_List_T list = nullptr;
  for (int i = k.nout - 1; i >= 0; i--) {
    const int32_t cell = cells[(size_t)i];
    if (cell >= 0) {  // the path's own cell (List_push_existing)
      RefList* l = incells[(size_t)(cell & (GSNAPDP_S3_CELL_DISALLOWED - 1))];
      ((RefPair*)l->first)->disallowedp = (cell & GSNAPDP_S3_CELL_DISALLOWED) ? 1 : 0;
      l->rest = (RefList*)list;
      list = (gsnapdp_List_T)l;
    } else {
      const gsnapdp_s3_pair& p = news[(size_t)(-1 - cell)];
      if (p.flags & GSNAPDP_S3_GAPP) {
        list = Pairpool_push_gapholder(list, pairpool, p.queryjump, p.genomejump,
                                       (p.flags & GSNAPDP_S3_KNOWNGAPP) ? 1 : 0);
        ((RefPair*)((RefList*)list)->first)->comp = p.comp;  // a microexon's gapchar (dynprog.c:6991)
      } else {
        list = Pairpool_push(list, pairpool, p.querypos, p.genomepos, p.cdna, p.comp, p.genome, p.dynprogindex);
      }
      // a pair an earlier fill of this call made and a later genome gap peeled
      // and put back keeps disallowedp = true (stage3.c:5873-5880); both pushes
      // start it false (pairpool.c:212, :400)
      ((RefPair*)((RefList*)list)->first)->disallowedp = (p.flags & GSNAPDP_S3_DISALLOWED) ? 1 : 0;
    }
  }
  return list;
}

}  // namespace

extern "C" {

// build_pairs_introns (stage3.c:7735-7901), the reference's static function with
// its signature (non-PMAP, non-WASTE), for a stage3.c that calls it here
// (:8766, :8865): the path goes through gsnapdp_stage3_pass (every gap filled
// on the GPU, the peels and accept rules on the host).  The genome is the
// context's (genome / genomicseg_ptr unused).
gsnapdp_List_T Gsnapdp_build_pairs_introns(
    gsnapdp_bool* shiftp, gsnapdp_bool* incompletep, int* nintrons, int* nnonintrons, int* intronlen,
    int* nonintronlen, int* dynprogindex_minor, int* dynprogindex_major, gsnapdp_List_T path, int chrnum,
    gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genome_T /*genome*/, int querylength, int genomiclength, char* queryseq_ptr, char* queryuc_ptr,
    char* /*genomicseg_ptr*/, char* /*genomicuc_ptr*/, gsnapdp_bool use_genomicseg_p, int cdna_direction,
    gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, int maxpeelback, int nullgap, int extramaterial_paired,
    int extraband_single, int extraband_paired, double defect_rate, int close_indels_mode,
    gsnapdp_Pairpool_T pairpool, gsnapdp_Dynprog_T dynprogL, gsnapdp_Dynprog_T dynprogM,
    gsnapdp_Dynprog_T dynprogR, gsnapdp_bool finalp) {
  if (use_genomicseg_p) fatal("build_pairs_introns on a genomic segment is not served by the batched pass");
  gsnapdp_s3_call k;
  memset(&k, 0, sizeof(k));
  k.pass = GSNAPDP_S3_INTRONS;
  k.querylength = querylength;
  k.chroffset = chroffset;
  k.chrhigh = chrhigh;
  k.chrpos = chrpos;
  k.chrnum = chrnum;
  k.genomiclength = genomiclength;
  k.cdna_direction = cdna_direction;
  k.watsonp = watsonp ? 1 : 0;
  k.jump_late_p = jump_late_p ? 1 : 0;
  k.finalp = finalp ? 1 : 0;
  k.maxpeelback = maxpeelback;
  k.nullgap = nullgap;
  k.extramaterial_paired = extramaterial_paired;
  k.extraband_single = extraband_single;
  k.extraband_paired = extraband_paired;
  k.close_indels_mode = close_indels_mode;
  k.defect_rate = defect_rate;
  const Dynprog* dp[3] = {(const Dynprog*)dynprogL, (const Dynprog*)dynprogM, (const Dynprog*)dynprogR};
  for (int i = 0; i < 3; i++) {
    k.maxlength1[i] = dp[i]->maxlength1;
    k.maxlength2[i] = dp[i]->maxlength2;
  }
  k.in_minor = *dynprogindex_minor;
  k.in_major = *dynprogindex_major;
  k.in_nintrons = *nintrons;
  k.in_nnonintrons = *nnonintrons;
  k.in_intronlen = *intronlen;
  k.in_nonintronlen = *nonintronlen;
  // Stage3_setup's flags as gmap derives them from Dynprog_setup's (gmap.c:3828-3849)
  k.novelsplicingp = g.novelsplicingp ? 1 : 0;
  k.splicingp = (g.novelsplicingp || g.splicing_iit) ? 1 : 0;
  // the splicing IIT of Dynprog_setup, asked through the host's own iit-read
  // functions (every genome-gap window's known-site record)
  gsnapdp_List_T list = pass_one(k, path, queryseq_ptr, queryuc_ptr, pairpool, g.iit ? host_iit() : nullptr,
                                 "build_pairs_introns");
  *shiftp = k.shiftp ? 1 : 0;
  *incompletep = k.incompletep ? 1 : 0;
  *nintrons = k.out_nintrons;
  *nnonintrons = k.out_nnonintrons;
  *intronlen = k.out_intronlen;
  *nonintronlen = k.out_nonintronlen;
  *dynprogindex_minor = k.out_minor;
  *dynprogindex_major = k.out_major;
  return list;
}

// build_pairs_singles (stage3.c:7454-7583), passes 2A / 2C / 7C of path_compute
// (:8671, :8700, :8938), with the reference's signature (non-PMAP, non-WASTE):
// every single gap (queryjump <= nullgap, neither a cDNA insertion nor an
// intron) is filled by traverse_single_gap (forcep false) in the batched pass;
// the query is the whole NUL-terminated query (Sequence_fullpointer).
gsnapdp_List_T Gsnapdp_build_pairs_singles(int* dynprogindex, gsnapdp_List_T path, gsnapdp_Genomicpos_T chroffset,
                                           gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
                                           gsnapdp_Genomicpos_T genomiclength, char* queryseq_ptr,
                                           char* queryuc_ptr, char* /*genomicseg_ptr*/, char* /*genomicuc_ptr*/,
                                           int cdna_direction, gsnapdp_bool watsonp, gsnapdp_bool jump_late_p,
                                           int maxpeelback, int nullgap, int extraband_single, double defect_rate,
                                           int close_indels_mode, gsnapdp_Pairpool_T pairpool,
                                           gsnapdp_Dynprog_T dynprogM) {
  gsnapdp_s3_call k;
  memset(&k, 0, sizeof(k));
  k.pass = GSNAPDP_S3_SINGLES;
  k.querylength = (int32_t)strlen(queryseq_ptr);
  k.chroffset = chroffset;
  k.chrhigh = chrhigh;
  k.chrpos = chrpos;
  k.genomiclength = (int32_t)genomiclength;
  k.cdna_direction = cdna_direction;
  k.watsonp = watsonp ? 1 : 0;
  k.jump_late_p = jump_late_p ? 1 : 0;
  k.maxpeelback = maxpeelback;
  k.nullgap = nullgap;
  k.extraband_single = extraband_single;
  k.close_indels_mode = close_indels_mode;
  k.defect_rate = defect_rate;
  for (int i = 0; i < 3; i++) {
    k.maxlength1[i] = ((const Dynprog*)dynprogM)->maxlength1;
    k.maxlength2[i] = ((const Dynprog*)dynprogM)->maxlength2;
  }
  k.in_minor = *dynprogindex;
  gsnapdp_List_T list =
      pass_one(k, path, queryseq_ptr, queryuc_ptr, pairpool, nullptr, "build_pairs_singles");
  *dynprogindex = k.out_minor;
  return list;
}

}  // extern "C"

namespace {

// the arguments build_pairs_end5 / build_path_end3 share (extendp; extend_ending5
// / extend_ending3, stage3.c:6587-6719 / :6906-7041)
void end_call(gsnapdp_s3_call& k, int pass, gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
              gsnapdp_Genomicpos_T chrpos, int querylength, int genomiclength, int cdna_direction,
              gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, int maxpeelback, int nullgap, int extramaterial_end,
              int extraband_end, double defect_rate, gsnapdp_Dynprog_T dynprog, gsnapdp_Endalign_T endalign,
              int minor) {
  memset(&k, 0, sizeof(k));
  k.pass = pass;
  k.querylength = querylength;
  k.chroffset = chroffset;
  k.chrhigh = chrhigh;
  k.chrpos = chrpos;
  k.genomiclength = genomiclength;
  k.cdna_direction = cdna_direction;
  k.watsonp = watsonp ? 1 : 0;
  k.jump_late_p = jump_late_p ? 1 : 0;
  k.maxpeelback = maxpeelback;
  k.nullgap = nullgap;
  k.extramaterial_end = extramaterial_end;
  k.extraband_end = extraband_end;
  k.defect_rate = defect_rate;
  k.endalign = (int32_t)endalign;
  for (int i = 0; i < 3; i++) {
    k.maxlength1[i] = ((const Dynprog*)dynprog)->maxlength1;
    k.maxlength2[i] = ((const Dynprog*)dynprog)->maxlength2;
  }
  k.in_minor = minor;
}

}  // namespace

extern "C" {

// build_pairs_end5 (stage3.c:7351-7450), passes 8, 9a and 10 of path_compute
// (:8966, :9036, :9167; path_trim :9660, :9722), with the reference's signature
// (non-GSNAP, non-PMAP):
// the 5' extension's Dynprog_end5_gap in the batched pass.  extendp only (the
// distalmedial branch is unused, :7420); without splice sites (Dynprog_end5_known
// is the splice-site branch of QUERYEND_GAP, :6651).
gsnapdp_List_T Gsnapdp_build_pairs_end5(
    gsnapdp_bool* knownsplicep, int* ambig_end_length_5, gsnapdp_Splicetype_T* /*ambig_splicetype_5*/,
    gsnapdp_bool* chop_exon_p, int* dynprogindex_minor, gsnapdp_List_T pairs, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos, int genomiclength,
    gsnapdp_Genomicpos_T /*knownsplice_limit_low*/, gsnapdp_Genomicpos_T /*knownsplice_limit_high*/,
    char* queryseq_ptr, char* queryuc_ptr, char* /*genomicseg_ptr*/, char* /*genomicuc_ptr*/, int cdna_direction,
    gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, int maxpeelback, int /*maxpeelback_distalmedial*/, int nullgap,
    int extramaterial_end, int extraband_end, double defect_rate, gsnapdp_Pairpool_T pairpool,
    gsnapdp_Dynprog_T dynprogR, gsnapdp_bool extendp, gsnapdp_Endalign_T endalign) {
  if (!extendp) fatal("build_pairs_end5: distalmedial_ending5 (extendp false) is not served");
  if (g.splicesites && endalign == GSNAPDP_QUERYEND_GAP)
    fatal("build_pairs_end5: Dynprog_end5_known (splice sites) is not served by the batched pass");
  *ambig_end_length_5 = 0;
  if (!pairs || ((const RefPair*)((RefList*)pairs)->first)->querypos < 0) return nullptr;  // :7372-7390
  gsnapdp_s3_call k;
  end_call(k, GSNAPDP_S3_END5, chroffset, chrhigh, chrpos, (int)strlen(queryseq_ptr), genomiclength, cdna_direction,
           watsonp, jump_late_p, maxpeelback, nullgap, extramaterial_end, extraband_end, defect_rate, dynprogR,
           endalign, *dynprogindex_minor);
  gsnapdp_List_T list = pass_one(k, pairs, queryseq_ptr, queryuc_ptr, pairpool, nullptr, "build_pairs_end5");
  *chop_exon_p = 0;
  *knownsplicep = 0;
  *dynprogindex_minor = k.out_minor;
  return list;
}

// build_path_end3 (stage3.c:7236-7347), the 3' counterpart (:8990, :9088, :9190,
// :9683, :9744)
gsnapdp_List_T Gsnapdp_build_path_end3(
    gsnapdp_bool* knownsplicep, int* ambig_end_length_3, gsnapdp_Splicetype_T* /*ambig_splicetype_3*/,
    gsnapdp_bool* chop_exon_p, int* dynprogindex_minor, gsnapdp_List_T path, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos, int querylength, int genomiclength,
    gsnapdp_Genomicpos_T /*knownsplice_limit_low*/, gsnapdp_Genomicpos_T /*knownsplice_limit_high*/,
    char* queryseq_ptr, char* queryuc_ptr, char* /*genomicseg_ptr*/, char* /*genomicuc_ptr*/, int cdna_direction,
    gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, int maxpeelback, int /*maxpeelback_distalmedial*/, int nullgap,
    int extramaterial_end, int extraband_end, double defect_rate, gsnapdp_Pairpool_T pairpool,
    gsnapdp_Dynprog_T dynprogL, gsnapdp_bool extendp, gsnapdp_Endalign_T endalign) {
  if (!extendp) fatal("build_path_end3: distalmedial_ending3 (extendp false) is not served");
  if (g.splicesites && endalign == GSNAPDP_QUERYEND_GAP)
    fatal("build_path_end3: Dynprog_end3_known (splice sites) is not served by the batched pass");
  *ambig_end_length_3 = 0;
  if (!path || ((const RefPair*)((RefList*)path)->first)->querypos < 0) return nullptr;  // :7257-7274
  gsnapdp_s3_call k;
  end_call(k, GSNAPDP_S3_END3, chroffset, chrhigh, chrpos, querylength, genomiclength, cdna_direction, watsonp,
           jump_late_p, maxpeelback, nullgap, extramaterial_end, extraband_end, defect_rate, dynprogL, endalign,
           *dynprogindex_minor);
  gsnapdp_List_T list = pass_one(k, path, queryseq_ptr, queryuc_ptr, pairpool, nullptr, "build_path_end3");
  *chop_exon_p = 0;
  *knownsplicep = 0;
  *dynprogindex_minor = k.out_minor;
  return list;
}

// build_dual_breaks (stage3.c:7149-7232), pass 5 of path_compute (:8831): a
// dual break solvable as a single gap runs traverse_single_gap (forcep) in the
// batched pass; one that is not calls the host program's own stage 2 through
// the pass's stage-2 callback, with this call's oligoindices and pools.
gsnapdp_List_T Gsnapdp_build_dual_breaks(
    gsnapdp_bool* dual_break_p, int* dynprogindex_minor, gsnapdp_List_T path, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos, gsnapdp_Genomicpos_T genomiclength,
    char* queryseq_ptr, char* queryuc_ptr, char* genomicseg_ptr, char* genomicuc_ptr, int cdna_direction,
    gsnapdp_bool watsonp, int genestrand, gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool,
    gsnapdp_Dynprog_T dynprogM, int maxpeelback, void* oligoindices_minor, int noligoindices_minor, void* diagpool,
    int sufflookback, int nsufflookback, int maxintronlen_bound, int extraband_single, double defect_rate,
    int close_indels_mode) {
  gsnapdp_s3_call k;
  memset(&k, 0, sizeof(k));
  k.pass = GSNAPDP_S3_DUALBREAKS;
  k.querylength = (int32_t)strlen(queryseq_ptr);
  k.chroffset = chroffset;
  k.chrhigh = chrhigh;
  k.chrpos = chrpos;
  k.genomiclength = (int32_t)genomiclength;
  k.cdna_direction = cdna_direction;
  k.watsonp = watsonp ? 1 : 0;
  k.jump_late_p = jump_late_p ? 1 : 0;
  k.maxpeelback = maxpeelback;
  k.extraband_single = extraband_single;
  k.close_indels_mode = close_indels_mode;
  k.defect_rate = defect_rate;
  for (int i = 0; i < 3; i++) {
    k.maxlength1[i] = ((const Dynprog*)dynprogM)->maxlength1;
    k.maxlength2[i] = ((const Dynprog*)dynprogM)->maxlength2;
  }
  k.in_minor = *dynprogindex_minor;
  Stage2Args a = {queryseq_ptr, queryuc_ptr, genomicseg_ptr, genomicuc_ptr, genestrand, watsonp ? 1 : 0,
                  oligoindices_minor, noligoindices_minor, pairpool, diagpool, sufflookback, nsufflookback,
                  maxintronlen_bound};
  k.invocation = stage2_register(&a);
  gsnapdp_List_T list = pass_one(k, path, queryseq_ptr, queryuc_ptr, pairpool, nullptr, "build_dual_breaks");
  stage2_unregister(k.invocation);
  *dual_break_p = k.shiftp ? 1 : 0;
  *dynprogindex_minor = k.out_minor;
  return list;
}

// build_pairs_dualintrons (stage3.c:7592-7733), pass 3b of path_compute
// (:8746): every short exon Smooth_pairs_by_size marked between two introns is
// weighed by traverse_dual_genome_gap (:5980-6364) -- one intron, two, or one
// of them -- with its Dynprog_genome_gap windows in the batched pass.
gsnapdp_List_T Gsnapdp_build_pairs_dualintrons(
    int* dynprogindex, gsnapdp_List_T path, int chrnum, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos, int genomiclength, char* queryseq_ptr,
    char* queryuc_ptr, char* /*genomicseg_ptr*/, char* /*genomicuc_ptr*/, gsnapdp_bool use_genomicseg_p,
    int cdna_direction, gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, int maxpeelback, int nullgap,
    int extramaterial_paired, int extraband_paired, double defect_rate, gsnapdp_Pairpool_T pairpool,
    gsnapdp_Dynprog_T dynprogL, gsnapdp_Dynprog_T dynprogR) {
  if (use_genomicseg_p) fatal("build_pairs_dualintrons on a genomic segment is not served by the batched pass");
  gsnapdp_s3_call k;
  memset(&k, 0, sizeof(k));
  k.pass = GSNAPDP_S3_DUALINTRONS;
  k.querylength = (int32_t)strlen(queryseq_ptr);
  k.chroffset = chroffset;
  k.chrhigh = chrhigh;
  k.chrpos = chrpos;
  k.chrnum = chrnum;
  k.genomiclength = genomiclength;
  k.cdna_direction = cdna_direction;
  k.watsonp = watsonp ? 1 : 0;
  k.jump_late_p = jump_late_p ? 1 : 0;
  k.maxpeelback = maxpeelback;
  k.nullgap = nullgap;
  k.extramaterial_paired = extramaterial_paired;
  k.extraband_paired = extraband_paired;
  k.defect_rate = defect_rate;
  const Dynprog* dp[3] = {(const Dynprog*)dynprogL, (const Dynprog*)dynprogL, (const Dynprog*)dynprogR};
  for (int i = 0; i < 3; i++) {
    k.maxlength1[i] = dp[i]->maxlength1;
    k.maxlength2[i] = dp[i]->maxlength2;
  }
  k.in_major = *dynprogindex;
  k.novelsplicingp = g.novelsplicingp ? 1 : 0;  // Stage3_setup's flags (gmap.c:3828-3849)
  k.splicingp = (g.novelsplicingp || g.splicing_iit) ? 1 : 0;
  gsnapdp_List_T list = pass_one(k, path, queryseq_ptr, queryuc_ptr, pairpool, g.iit ? host_iit() : nullptr,
                                 "build_pairs_dualintrons");
  *dynprogindex = k.out_major;
  return list;
}

double Maxent_hr_donor_prob(gsnapdp_Genomicpos_T splice_pos, gsnapdp_Genomicpos_T chroffset) {
  return maxent_one(GSNAPDP_DONOR, splice_pos, chroffset);
}
double Maxent_hr_acceptor_prob(gsnapdp_Genomicpos_T splice_pos, gsnapdp_Genomicpos_T chroffset) {
  return maxent_one(GSNAPDP_ACCEPTOR, splice_pos, chroffset);
}
double Maxent_hr_antidonor_prob(gsnapdp_Genomicpos_T splice_pos, gsnapdp_Genomicpos_T chroffset) {
  return maxent_one(GSNAPDP_ANTIDONOR, splice_pos, chroffset);
}
double Maxent_hr_antiacceptor_prob(gsnapdp_Genomicpos_T splice_pos,
                                   gsnapdp_Genomicpos_T chroffset) {
  return maxent_one(GSNAPDP_ANTIACCEPTOR, splice_pos, chroffset);
}

}  // extern "C"
