// gsnapdp_band.h -- the register-band machinery shared by k_fill (single
// gaps, gsnapdp_kernels.hip) and k_gband (genome-gap flanks, gsnapdp_gband.hip):
// the column genome stream, the 16-bit cell values, the lane shifts, the LDS
// rings and the backward traceback sweep over the per-wave direction scratch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "gsnapdp_device.h"
#include "gsnapdp_internal.h"

#ifndef AS_GLOBAL
#define AS_GLOBAL __attribute__((address_space(1)))
#define AS_LDS __attribute__((address_space(3)))
#endif

namespace gsnapdp {

// ------------------------------------------------------------------ k_fill
// Per-lane column genome stream: class of column c for the window, branch
// free.  pos(c) = P0 + PS*c in reference uint32 arithmetic (get_genomic_nt).
struct ColStream {
  uint32_t P0;
  int PS;        // +1 / -1
  int cvlo, cvhi;  // columns whose genomicpos is inside [0, genomiclength)
  int xorc;      // 0 watson, 3 crick (complement of the 2-bit code)
  __device__ inline void init(const Lane& L) {
    const int gstep = L.gstep;
    if (L.watson) {
      P0 = L.base + (uint32_t)(L.g0 - gstep);
      PS = gstep;
    } else {
      P0 = L.base + (uint32_t)(L.glen - 1) - (uint32_t)(L.g0 - gstep);
      PS = -gstep;
    }
    if (gstep > 0) {
      cvlo = 1 - L.g0;
      cvhi = L.glen - L.g0;
    } else {
      cvlo = L.g0 + 2 - L.glen;
      cvhi = L.g0 + 1;
    }
    if (L.allstar) {
      cvlo = 1 << 30;
      cvhi = -(1 << 30);
    }
    xorc = L.watson ? 0 : 3;
  }
  __device__ inline int cls(const uint32_t* __restrict__ blocks, uint64_t nwords, int c) const {
    const uint32_t pos = P0 + (uint32_t)(PS * c);
    const uint64_t ptr = (uint64_t)(pos >> 5) * 3u;
    const bool inr = c >= cvlo && c <= cvhi;
    const bool ing = ptr + 2 < nwords;
    const uint64_t p = (inr && ing) ? ptr : 0;
    const uint32_t bit = pos & 31u;
    const uint32_t fl = blocks[p + 2];
    const uint32_t word = blocks[p + (bit < 16 ? 1 : 0)];
    const int code = (int)((word >> ((bit & 15u) * 2u)) & 3u) ^ xorc;
    const bool isn = !ing || ((fl >> bit) & 1u);
    return !inr ? 5 : (isn ? 4 : code);
  }
};

#ifndef GSNAPDP_FILL_WAVES
#define GSNAPDP_FILL_WAVES 3  // k_fill waves per SIMD (register budget 512 / waves; 4 measured 0.6 % slower on C3, 6 % on C2)
#endif
constexpr int FILL_SC_BIAS = 6;  // -2 * SINGLE_EXTEND (dynprog.c:222)
#ifndef GSNAPDP_TB_AHEAD
#define GSNAPDP_TB_AHEAD 1
#endif
constexpr int TB_AHEAD = GSNAPDP_TB_AHEAD;  // traceback prefetch distance, in 4-column groups

// k_fill's LDS profile word: each signed 4-bit pairdistance nibble s becomes
// the unsigned nibble s + 6 (s in -5..3, so 1..9); match bits unchanged.
// END_SC_BIAS: the end gaps' ENDQ table (extend -1) folds -2 * END_EXTEND =
// +2 instead and stays signed (-3..5, read with a signed bfe).
constexpr int END_SC_BIAS = 2;  // -2 * END_EXTEND (dynprog.c:245)
__device__ inline uint32_t fill_profile_word(uint32_t w, int bias = FILL_SC_BIAS) {
  uint32_t o = w & 0xFF000000u;
#pragma unroll
  for (int g = 0; g < 6; g++) {
    const int n = (int)((w >> (4 * g)) & 0xFu);
    const int sn = n >= 8 ? n - 16 : n;
    o |= (uint32_t)((sn + bias) & 0xF) << (4 * g);
  }
  return o;
}
constexpr int UTAB = 4 * 128;  // LDS profile: 4 x 128 pairdistance words, then 256 uppercase words
constexpr int MLUT = UTAB + 256;  // then 32 uint64: the 5 match bits of a profile word spread to bit 7 of bytes 0..4
constexpr int SPROF_WORDS = MLUT + 64;
__host__ __device__ constexpr uint64_t spread_match(uint32_t m5) {
  uint64_t x = 0;
  for (int k = 0; k < 5; k++)
    if ((m5 >> k) & 1u) x |= (uint64_t)1 << (8 * k + 7);
  return x;
}

// f(integral_constant<int, U>) for U in the sequence, in order
template <int... U, class F>
__device__ inline void unroll_seq(std::integer_sequence<int, U...>, F&& f) {
  (f(std::integral_constant<int, U>()), ...);
}
// k_fill's cell values.  By default they are 16-bit: value + FV_BIAS, NEG-like
// values from FV_NEG up, all zero-extended in 32-bit registers, so the maxima
// are v_max_u16 (twice the issue rate of v_max_i32 on gfx950; 16-bit VOP2
// results zero bits 16-31) while sums and differences stay 32-bit adds.
// In-band reachable values lie in [2*open + 1, 9 * steps] (offset
// coordinates, open >= -12 for the single gaps k_fill serves), NEG-like ones
// in [FV_NEG + open, FV_NEG + 9 * steps]; with at most 688 steps both ranges
// stay apart and inside 0..65535 (static_assert below).
#ifndef GSNAPDP_FILL32
using FV = uint32_t;
constexpr uint32_t FV_NEG = 1024u;
constexpr uint32_t FV_BIAS = 16384u;
__device__ inline FV fv_max(FV a, FV b) {
  FV d;
  asm("v_max_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ inline FV fv_min(FV a, uint32_t b) {  // 16-bit min (b's low half)
  FV d;
  asm("v_min_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// min(x, bits 16..31 of w) (both 16-bit), the upper half of the result zeroed
__device__ inline FV fv_cap_hi(FV x, uint32_t w) {
  FV d;
  asm("v_min_u16_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1"
      : "=v"(d)
      : "v"(x), "v"(w));
  return d;
}
static_assert(FV_NEG >= 12 && FV_NEG + 9u * 688u < FV_BIAS - 2u * 12u &&
                  FV_BIAS + 9u * 688u < 65536u && FAST_L2MAX + 48 <= 688,
              "16-bit k_fill value ranges");
// End gaps (ENDQ, open -12, extend -1): a diagonal step changes an offset value
// by pairdistance + 2 in -3..5, so values fall as well as rise.  Their NEG-like
// values start higher, at FV_NEG_END, and stay in [FV_NEG_END - 24 - 3*688,
// FV_NEG_END + 5*688], below the reachable [FV_BIAS - 24 - 3*688, FV_BIAS +
// 5*688], which stays under bit 15 (the live-row cap, k_fill).
constexpr uint32_t FV_NEG_END = 4096u;
static_assert(FV_NEG_END >= 24u + 3u * 688u && FV_NEG_END + 5u * 688u < FV_BIAS - 24u - 3u * 688u &&
                  FV_BIAS + 5u * 688u < 32768u,
              "16-bit k_fill end-gap value ranges");
#else
using FV = int;
constexpr int FV_NEG = NEG;
constexpr int FV_BIAS = 0;
constexpr int FV_NEG_END = NEG;
__device__ inline FV fv_max(FV a, FV b) { return max(a, b); }
__device__ inline FV fv_cap_hi(FV x, uint32_t) { return x; }  // (k_plan keeps end gaps off this build)
__device__ inline FV fv_min(FV a, uint32_t b) { return a; }
#endif
__device__ inline uint32_t push_sign(uint32_t acc, int d) {
  return __builtin_amdgcn_alignbit(acc, (uint32_t)d, 31u);  // (acc << 1) | (d < 0)
}
// the same register of lane-1 / lane+1 (rows of 16 lanes; groups never straddle rows)
__device__ inline int from_lane_above(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x111, 0xF, 0xF, true);  // row_shr:1
}
__device__ inline int from_lane_below(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x101, 0xF, 0xF, true);  // row_shl:1
}
// (a, b) = min((x, y) of lane-1, cap) as 16-bit values, one v_min_u16_dpp each
// where a DPP move and a select were two.  A lane without a source in its
// 16-lane row is not written (bound_ctrl off): a and b are loop-carried, so
// those lanes keep what they held (the caller starts them at a NEG-like
// value).  The s_nop covers the DPP read-after-VALU-write hazard (2 wait
// states), which the compiler does not see through inline asm.
__device__ inline void min2_from_lane_above(uint32_t& a, uint32_t& b, uint32_t x, uint32_t y, uint32_t cap) {
  asm("s_nop 1\n\t"
      "v_min_u16_dpp %0, %2, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_min_u16_dpp %1, %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf"
      : "+v"(a), "+v"(b)
      : "v"(x), "v"(y), "v"(cap));
}
__device__ inline void min2_from_lane_below(uint32_t& a, uint32_t& b, uint32_t x, uint32_t y, uint32_t cap) {
  asm("s_nop 1\n\t"
      "v_min_u16_dpp %0, %2, %4 row_shl:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_min_u16_dpp %1, %3, %4 row_shl:1 row_mask:0xf bank_mask:0xf"
      : "+v"(a), "+v"(b)
      : "v"(x), "v"(y), "v"(cap));
}

// A pointer every lane holds the same value of (a kernel argument passed down
// into a non-inlined function, which receives it in VGPRs): rebuilt from SGPRs,
// so that its loads and stores address it as a scalar base (global_* saddr,
// buffer resources) instead of per-lane 64-bit arithmetic.
template <class T>
__device__ inline T* wave_uniform(T* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return (T*)(((uint64_t)hi << 32) | lo);
}

// Per-wave LDS rings of k_fill (sizes per band class): for each window of the
// wave, the profile words of the rows its lanes' bottom slots will need and the
// genome classes of the columns they will need, staged RING_K columns at a time.
constexpr int RING_K = 16;
constexpr int pow2ceil(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}
template <int S, int LPW>
struct Rings {
  static constexpr int NG = 64 / LPW;
  static constexpr int SPAN = (LPW - 1) * (S - 1);  // rows between the group's bottom slots
  static constexpr int RR = pow2ceil(RING_K + SPAN);
  static constexpr int CR = pow2ceil(RING_K + LPW - 1);
  static constexpr int WORDS = NG * RR + (NG * CR + 3) / 4;
};
constexpr int RING_WORDS_MAX = 1280;  // max Rings<S,LPW>::WORDS over the classes (checked below)


// ---- traceback (dynprog.c:2611-2712) on lane 0 of each window group, as a
// backward sweep in which every lane visits the same column at the same time
// (a window waits until the sweep reaches its own start column).  The path's
// current diagonal (slot, owning lane, bit position) stays in registers, so a
// diagonal step costs a few ALU ops; the direction and match words of that
// lane arrive four columns per group, one group ahead.  VERT / HORIZ runs
// take the general path; a gap that moves the path to another lane's slots
// costs one dependent load.
//
// D / M: the wave's direction words and match bytes (column c's 64-lane row at
// c * 64, lane (j, g) at j * NG + g); (r, cstart): the start cell; maxC: the
// wave's largest start column (every lane of the wave computes it; the
// callers' other lanes have returned); JL: the fill's tie rule (its direction
// bits are stored complemented).  Adds to `tal` (npush: the HGAP gapholders
// only) and writes `ow`.
// The genome of a window's columns for the traceback's intron test: the packed
// genome, or (seg != nullptr) the caller's segment, genome position p at seg[p - g0].
struct SegCls {
  const unsigned char* seg;
  int g0;
};
#ifdef TB_PROF
// diagnostic builds: sweep counters (0 sweeps, 1 groups, 2 groups some lane
// could not bulk-step, 3 lane-columns stepped one by one, 4/5 fill / trace cycles)
__device__ unsigned long long tb_prof[8];
#define TB_COUNT(k, v)                                                      \
  do {                                                                      \
    if ((threadIdx.x & 63) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63)) \
      atomicAdd(&tb_prof[k], (unsigned long long)(v));                      \
  } while (0)
#else
#define TB_COUNT(k, v) \
  do {                 \
  } while (0)
#endif
// MATCH = false (k_fill): no match bytes; every diagonal step inside the
// window's genome is counted in nmismatches, and k_count splits the total into
// matches and mismatches afterwards from the op stream.
// PL: the bit stride of the direction planes in a lane's word (S: packed, the
// k_gband fills; 8: one byte per plane, k_fill's v_perm_b32 assembly)
template <int S, int LPW, bool MATCH = true, int PL = S>
__device__ inline void band_traceback(const uint32_t* __restrict__ D, const uint8_t* __restrict__ M,
                                      int g, int r, int cstart, int maxC, int lband, int rband,
                                      int stop, int cvlo, int cvhi, int JL, const Lane& L,
                                      const uint32_t* __restrict__ blocks, uint64_t nwords,
                                      Tally& tal, OpWriter& ow, const SegCls& sg = SegCls{nullptr, 0}) {
  constexpr int WMAX = S * LPW;
  constexpr int NG = 64 / LPW;
  enum { T_WAIT = 0, T_DIAG = 1, T_VERT = 2, T_HORIZ = 3, T_DONE = 4 };
  int st = T_WAIT;
  int dist = 0;
  int jj = 0, pb = 0;  // DIAG: lane holding the path's diagonal, bit of its slot in each plane
  const uint32_t jlbit = JL ? 1u : 0u;
  const int wband = lband + rband;
  const uint32_t* Dg = D + g;
  const uint8_t* Mg = M + g;
  auto set_diag = [&](int rr, int cc) {
    const int sg = stop + rr - cc + rband;
    const int sgc = sg < 0 ? 0 : (sg >= WMAX ? WMAX - 1 : sg);  // out of band: DONE next
    jj = sgc / S;
    pb = S - 1 - (sgc - jj * S);
  };
  auto ldw = [&](int cc, int jw) -> uint32_t { return Dg[(size_t)cc * 64 + jw * NG]; };
  auto ldm = [&](int cc, int jw) -> uint32_t { return Mg[(size_t)cc * 64 + jw * NG]; };
  struct Grp {
    uint32_t w[4], m[4];
    int jw;
  };
  auto fetch_group = [&](Grp& x, int G, int jw) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int cc = 4 * G + k;
      x.w[k] = ldw(cc, jw);
      if constexpr (MATCH) x.m[k] = ldm(cc, jw);
    }
    x.jw = jw;
  };
  auto column = [&](int c, uint32_t wk, uint32_t mk, int jw) {
    auto inb = [&](int rr) {
      const int d = rr - c + rband;
      return rr >= 1 && c >= 1 && d >= 0 && d <= wband;
    };
    auto plane_bit = [&](int rr, int plane) -> uint32_t {  // planes dE | dF | h1 | v1 from bit 0
      const int sg = stop + rr - c + rband;
      const int jr = sg / S, sl = sg - jr * S;
      const uint32_t x = (jr == jw) ? wk : ldw(c, jr);
      return ((x >> (plane * PL + S - 1 - sl)) & 1u) ^ jlbit;
    };
    if (st == T_WAIT && c == cstart) {
      st = T_DIAG;
      set_diag(r, c);
    }
    if (st == T_VERT) {  // gap2 chain in this column (add_queryskip, dynprog.c:2372)
      while (c == 0 ? (r >= 2 && r <= lband && r <= L.d.L1) : (inb(r) && plane_bit(r, 1))) {
        dist++;
        r--;
      }
      r--;
      ow.flush();
      ow.put(GSNAPDP_OP(GSNAPDP_OP_VSKIP, dist));
      tal.nopens++;
      tal.nindels += dist;
      st = T_DIAG;
      set_diag(r, c);
    }
    if (st == T_HORIZ) {  // gap1 chain, one column per step (add_genomeskip, dynprog.c:2416)
      const bool more = (r == 0) ? (c >= 2 && c <= rband && c <= L.d.L2) : (inb(r) && plane_bit(r, 0));
      if (more) {
        dist++;
      } else {
        // skipped columns c .. c+dist-1; the path lands in column c-1
        bool dashes = true;
        if (dist >= MICROINTRON_LENGTH) {
          const int cl = c, cr = c + dist - 1;
          const int gl = L.g0 + L.gstep * (cl - 1), gr = L.g0 + L.gstep * (cr - 1);
          const int lo = L.d.rev ? gr : gl, hi = L.d.rev ? gl : gr;
          auto cls = [&](int p) { return sg.seg ? seg_class(sg.seg[p - sg.g0]) : gclass(blocks, nwords, L, p); };
          const int l1 = cls(lo), l2 = cls(lo + 1);
          const int r2 = cls(hi - 1), r1 = cls(hi);
          dashes = intron_type_codes(l1, l2, r2, r1, L.cdna_direction) == 0;
        }
        ow.flush();
        ow.put(GSNAPDP_OP(dashes ? GSNAPDP_OP_HDASH : GSNAPDP_OP_HGAP, dist));
        if (dashes) {
          tal.nopens++;
          tal.nindels += dist;
        } else {
          tal.npush++;  // the HGAP gapholder (the other pushes follow from the counts)
        }
        st = T_DIAG;
        set_diag(r, c - 1);
      }
    } else if (st == T_DIAG) {
      if (!inb(r)) {
        st = T_DONE;
      } else {
        const uint32_t x = ((jj == jw) ? wk : ldw(c, jj)) >> pb;
        if (c >= cvlo && c <= cvhi) {  // not a '*' column (dynprog.c:2644)
          if constexpr (MATCH) {
            const uint32_t mb = (((jj == jw) ? mk : ldm(c, jj)) >> (S - 1 - pb)) & 1u;
            tal.nmatches += (int)mb;
            tal.nmismatches += 1 - (int)mb;
          } else {
            tal.nmismatches++;
          }
        }
        ow.run++;
        if (((x >> (3 * PL)) & 1u) ^ jlbit) {  // v1: VERT
          st = T_VERT;
          dist = 1;
        } else if (((x >> (2 * PL)) & 1u) ^ jlbit) {  // h1: HORIZ
          st = T_HORIZ;
          dist = 1;
        }
        r--;
      }
    }
  };
  // wave-uniform sweep from the wave's longest window down to column -1
  int G = maxC >> 2;
  TB_COUNT(0, 1);
  set_diag(r, cstart);
  // pre[0] is the group being visited, pre[1..TB_AHEAD] the next ones,
  // loaded TB_AHEAD groups ahead of their visit (global scratch latency)
  Grp pre[TB_AHEAD + 1];
#pragma unroll
  for (int i = 0; i <= TB_AHEAD; i++) fetch_group(pre[i], G - i >= 0 ? G - i : 0, jj);
  Grp& ga = pre[0];
  const uint32_t invall = JL ? 0xFFFFFFFFu : 0u;
  // one iteration per 4-column group G; its columns are visited one by one
  // only when some lane of the wave cannot take the group in one bulk step
  for (; G >= 0; G--) {
    const int chi = min(4 * G + 3, maxC);  // the first group may be partial
    bool fast4 = false;
    if (chi == 4 * G + 3) {
      // Four diagonal steps at once: the path stays on its diagonal through
      // columns c .. c-3 (no v1/h1 there), inside the band and the query, and
      // the four columns are all inside or all outside the window's genome.
      const int c = chi;
      const int dd = (S - 1 - pb) + jj * S - stop;  // the diagonal's offset in the band
      fast4 = st == T_DIAG && jj == ga.jw && r >= 4 && c >= 4 && dd >= 0 && dd <= wband;
      if (fast4) {
        const uint32_t x0 = (ga.w[0] ^ invall) >> pb, x1 = (ga.w[1] ^ invall) >> pb;
        const uint32_t x2 = (ga.w[2] ^ invall) >> pb, x3 = (ga.w[3] ^ invall) >> pb;
        const bool inside = c - 3 >= cvlo && c <= cvhi;
        const bool outside = c < cvlo || c - 3 > cvhi;
        const uint32_t vh = (1u << (2 * PL)) | (1u << (3 * PL));  // h1 and v1 of this slot
        fast4 = ((x0 | x1 | x2 | x3) & vh) == 0u && (inside || outside);
        if (fast4) {
          if (!MATCH && inside) {
            tal.nmismatches += 4;
          } else if (inside) {
            const int mb = S - 1 - pb;  // match bit of the diagonal's slot
            const int mcount = (int)(((ga.m[0] >> mb) & 1u) + ((ga.m[1] >> mb) & 1u) +
                                     ((ga.m[2] >> mb) & 1u) + ((ga.m[3] >> mb) & 1u));
            tal.nmatches += mcount;
            tal.nmismatches += 4 - mcount;
          }
          ow.run += 4;
          r -= 4;
        }
      }
    }
    // lanes with nothing to do in this group: bulk-stepped, done, or still
    // waiting for their own start column
    const bool idle = fast4 || st == T_DONE || (st == T_WAIT && cstart < 4 * G);
    TB_COUNT(1, 1);
    if (__builtin_amdgcn_ballot_w64(!idle) != 0) {
      TB_COUNT(2, 1);
      TB_COUNT(3, __builtin_popcountll(__builtin_amdgcn_ballot_w64(!idle)));
      for (int c = chi; c >= 4 * G; c--) {
        const int k = c & 3;
        if (!fast4 && st != T_DONE && (st != T_WAIT || c == cstart)) {
          const uint32_t wk = k == 0 ? ga.w[0] : k == 1 ? ga.w[1] : k == 2 ? ga.w[2] : ga.w[3];
          const uint32_t mk = !MATCH ? 0u : k == 0 ? ga.m[0] : k == 1 ? ga.m[1] : k == 2 ? ga.m[2] : ga.m[3];
          column(c, wk, mk, ga.jw);
        }
      }
    }
    // leaving group G
    if (__builtin_amdgcn_ballot_w64(st != T_DONE) == 0) break;
#pragma unroll
    for (int i = 0; i < TB_AHEAD; i++) {
      pre[i] = pre[i + 1];
      // a gap moved the path to another lane: reload the groups already in flight
      if (G - 1 - i >= 0 && pre[i].jw != jj) fetch_group(pre[i], G - 1 - i, jj);
    }
    if (G - 1 - TB_AHEAD >= 0) fetch_group(pre[TB_AHEAD], G - 1 - TB_AHEAD, jj);  // predicted unchanged
  }
  if (st != T_DONE && st != T_WAIT) column(-1, 0u, 0u, -1);
  ow.flush();
}

}  // namespace gsnapdp
