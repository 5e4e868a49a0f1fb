// sdx_general.hip -- the general path: MU/MS messages and MC frames outside the fixed-layout
// kernels' contract (include/sdx.h "general path"), hand-written HIP for gfx950.
//
// k_pulses keeps a message as per-id position bitmaps, which needs single-character pattern ids
// (P0..P9) and <= 4096 pulses; k_mc keeps a frame's bits in LDS (<= 128 hex characters).  The
// reference has neither limit: it keys patterns by str(int(key[1:])) ("P10" is the two-character
// id "10", message_unsynced.py:28-35, message_synced.py:50-57), builds candidate targets by string
// concatenation (pattern_utils.py:120-130), matches MU with re.finditer over alternations of those
// strings (message_unsynced.py:146-200) and slices chunks by characters (:203-221; MS :172-189).
// This file restates that string semantics directly, one wave per message walking the bank in bank
// order (the order results and raises take in the reference), the 64 lanes sharing the wide steps:
//   * pattern_exists: candidates by the fp64 gap test, stable gap order, itertools.product order,
//     no id reused, first target string that occurs (str `in`);
//   * MU matching: Python sre's order for (?:S)((?:U1|U2|..){lmin,}(?:E1|..)?) -- leftmost start,
//     alternatives in order, greedy repetition that backtracks only while fewer than lmin units
//     matched (past lmin every continuation succeeds), then the first end key that matches;
//   * chunks, postDemodulation, padding, hex / bin formatting, modulematch: as the lane kernels
//     (sdx_device.h run_postdemo, dfa_accepts).
// Results: the message's list is counted in a first pass, reserved with one atomic pair and written
// in a second (deterministic) pass.  Messages this path takes are rare (the SIGNALduino firmware
// emits P0..P7 and short lines); throughput is not its goal, exactness is.
#include "sdx_mc.h"

#include <string>

namespace sdx {
int set_error(int code, const std::string& msg);  // sdx_kernels.hip
const void* bank_dev_ptr(const sdx_bank* b);
const sdx_bank_hdr* bank_hdr(const sdx_bank* b);
}  // namespace sdx

namespace sdxg {
using namespace sdx;

#define GD __device__ __attribute__((noinline))
#define GI __device__ __forceinline__

// SDX_GPROF (variant builds only, tools/prof_general.py): s_memtime cycles per phase of the MU walk,
// summed over items (lane 0 adds), and each pass-0 item's cycles in GenChunk.res
#ifdef SDX_GPROF
__device__ unsigned long long g_genprof[16];
#define GP_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define GP_ADD(slot, t0) \
  do { if (lane_id() == 0) atomicAdd(&g_genprof[slot], __builtin_amdgcn_s_memtime() - (t0)); } while (0)
#define GP_CNT(slot) \
  do { if (lane_id() == 0) atomicAdd(&g_genprof[slot], 1ull); } while (0)
#else
#define GP_T(v)
#define GP_ADD(slot, t0)
#define GP_CNT(slot)
#endif

constexpr int GP = SDX_GEN_MAXPAT, GID = SDX_GEN_IDSTR, GS = SDX_GEN_STRMAX, GREP = SDX_GEN_REPMAX;
constexpr long long GBUDGET = 1ll << 22;  // sre steps per repetition match (catastrophic backtracking)
constexpr int GSLACK = 512;               // per-message scratch beyond n: padding, postDemo prefixes, texts

struct Str {
  int len;
  uint8_t c[GS];
};

// the wave's small working set, in LDS (all lanes write the same values and read them back):
// dynamically indexed private arrays would live in scratch memory, at global-memory latency
struct Wk {
  Str str[8];                        // MU: S, U[3], E[3], the pex target; MS: K[4], E[3], the target
  uint8_t sym[8];                    // symbols of the unit / end strings
  uint8_t cand[SDX_MAXUNIQ][GP];     // pattern_exists candidates per unique value
  int cnt[SDX_MAXUNIQ], digit[SDX_MAXUNIQ];
  double gap[GP];
  uint8_t ch[GREP];                  // rep_match choice stack
  int ps[GREP];
};

struct Msg {
  Wk* wk;
  const uint8_t* d;
  int n;
  int npat;
  const uint8_t* ids;  // [GP][GID]
  const double* val;   // [GP]
  double nv[GP];       // round(P / clock, 1)
  const uint64_t* bm;  // per digit character c: bm[c * nwp + w] bit j = d[64w + j] == '0' + c
  int nwp;             // words per character bitmap (one zero word of padding)
  uint64_t* tb;        // the MU match tables (position bitmaps, mu_tables): LDS or the slot's scratch
  int nwt;             // words per table bitmap (three zero words of padding)
  uint8_t* ld;         // the LDS copy of the characters (nullptr: they do not fit), made by stage()
  int staged;          // 1 once the characters are in the LDS copy (m.d points there)
};

// The serial steps (sre fallback, chunk compares) read the message's characters: copy them to the LDS
// once per message, and only when a protocol gets past its key lookups (most items stop before).
GD void stage(Msg& m) {
  if (m.staged || !m.ld) return;
  const uint8_t* src = m.d;
  uint8_t* dst = m.ld;
  const int n = m.n;
  __syncthreads();
  for (int j = lane_id(); j < n; j += 64) dst[j] = src[j];
  m.d = dst;
  m.staged = 1;
  __syncthreads();
}

// MU match tables, one position bitmap each (bit p of word p >> 6), nwt = (n >> 6) + 3 words:
//   UA[a]   unit string a occurs at p (a < 3)
//   SA      the start string occurs at p
//   D0, D1  {p : (?:U0|U1|..){r} can match at p} for the round r (double buffer)
//   G0, G1  the same for the greedy path (first matching unit at every step)
constexpr int TB_ARRAYS = 8;
__host__ __device__ inline int tb_words(int n) { return (n >> 6) + 3; }
__host__ __device__ inline int64_t tb_bytes(int n) { return (int64_t)TB_ARRAYS * 8 * tb_words(n); }

// bits q .. q+63 of character c's occurrence bitmap (q >= 0; the padding word ends every row)
GI uint64_t bm_at(const Msg& m, int c, int q) {
  const uint64_t* r = m.bm + (size_t)c * m.nwp;
  const int w = q >> 6, o = q & 63;
  if (w >= m.nwp - 1) return 0ull;
  const uint64_t lo = r[w];
  return o ? (lo >> o) | (r[w + 1] << (64 - o)) : lo;
}

// str.find(s, from) over the bitmaps, the whole wave: lane l tests the 64 start positions of word
// w0 + l (one AND per character of s; pattern strings are digit strings, ids are str(int(key[1:]))),
// the lowest lane with a hit gives the position.  Called in wave-uniform control flow (every lane
// holds the same message state, k_general), so 4096 start positions go per step.
GD int find_bm(const Msg& m, int from, const Str& s) {
  if (s.len == 0) return from <= m.n ? from : -1;
  const int last = m.n - s.len;
  if (from < 0) from = 0;
  if (from > last) return -1;
  const int wf = from >> 6, wl = last >> 6, lane = lane_id();
  for (int w0 = wf; w0 <= wl; w0 += 64) {
    const int w = w0 + lane;
    uint64_t acc = 0;
    if (w <= wl) {
      acc = ~0ull;
      for (int i = 0; i < s.len && acc; ++i) acc &= bm_at(m, s.c[i] - '0', w * 64 + i);
      if (w == wf) acc &= ~0ull << (from & 63);
      if (w == wl && (last & 63) != 63) acc &= (1ull << ((last & 63) + 1)) - 1;
    }
    const uint64_t hit = ballot(acc != 0);
    if (hit) return bcast_i(acc ? w * 64 + ffs64(acc) : 0, ffs64(hit));
  }
  return -1;
}

// result sink: pass 1 counts, pass 2 writes at the reserved bases
struct Sink {
  bool write;
  int nrec;
  uint32_t nheap;
  sdx_result* rec;
  uint8_t* heap;
  uint32_t rbase, hbase, msg;
};

GI bool at(const uint8_t* d, int n, int p, const uint8_t* s, int len) {
  if (p < 0 || p + len > n) return false;
  for (int i = 0; i < len; ++i)
    if (d[p + i] != s[i]) return false;
  return true;
}
GI bool str_eq(const Str& a, const Str& b, int blen) {  // a == b[:blen]
  if (a.len != blen) return false;
  for (int i = 0; i < blen; ++i)
    if (a.c[i] != b.c[i]) return false;
  return true;
}
GI void str_set(Str& a, const Str& b, int blen) {  // a = b[:blen]
  for (int i = 0; i < blen; ++i) a.c[i] = b.c[i];
  a.len = blen;
}
// pattern_exists(search, patterns, d[base:]) (pattern_utils.py:34-136): 1 found (*out = the target
// string), 0 = -1, -1 = the target would exceed SDX_GEN_STRMAX characters (contract)
GD int pex(const Msg& m, const sdx_patspec* sp, int base, Str* out) {
  const int slen = sp->len, nu = sp->nuniq;
  auto& cand = m.wk->cand;
  int* cnt = m.wk->cnt;
  int* digit = m.wk->digit;
  double* gap = m.wk->gap;
  int total = 1;
  for (int u = 0; u < nu; ++u) {
    const double uv = sp->uval[u], tol = sp->utol[u];
    int c = 0;
    for (int k = 0; k < m.npat; ++k) {
      const double g = fabs(m.nv[k] - uv);
      if (g <= 0.001 || g <= tol) {  // (:70-72)
        int j = c++;                 // stable sort by gap (:76-78): move past strictly larger gaps only
        while (j > 0 && gap[j - 1] > g) {
          gap[j] = gap[j - 1];
          cand[u][j] = cand[u][j - 1];
          --j;
        }
        gap[j] = g;
        cand[u][j] = (uint8_t)k;
      }
    }
    if (c == 0) return 0;  // (:73-75)
    cnt[u] = c;
    total *= c;
    if (total > 10000) return 0;  // (:88-95): the product only grows
  }
  for (int u = 0; u < SDX_MAXUNIQ; ++u) digit[u] = 0;
  for (int it = 0; it < total; ++it) {
    uint32_t used = 0;
    bool dup = false;
    for (int u = 0; u < nu; ++u) {
      const int k = cand[u][digit[u]];
      if ((used >> k) & 1u) dup = true;
      used |= 1u << k;
    }
    if (!dup) {  // (:111-113); the target is built in *out
      Str& t = *out;
      int tl = 0;
      for (int s = 0; s < slen; ++s) {
        const int u = sp->uidx[s];
        const int k = cand[u][digit[u]];
        const int L = m.ids[k * GID];
        if (tl + L > GS) return -1;
        for (int j = 0; j < L; ++j) t.c[tl++] = m.ids[k * GID + 1 + j];
      }
      t.len = tl;
      if (find_bm(m, base, t) >= 0) return 1;  // (:133-134)
    }
    for (int u = nu - 1; u >= 0; --u) {  // itertools.product: the last list varies fastest
      if (digit[u] + 1 < cnt[u]) {
        digit[u]++;
        break;
      }
      digit[u] = 0;
    }
  }
  return 0;
}

// (?:U0|U1|..){lmin,} at q in Python sre order: alternatives in order, another iteration before
// stopping; a dead end below lmin iterations backtracks to the latest choice with a further
// alternative.  Returns the end of the repetition or -1; *over on the step budget / depth limit.
GD int rep_match(const uint8_t* d, int n, int q, const Str* U, int nu, int lmin, bool* over, uint8_t* ch, int* ps) {
  long long steps = 0;
  if (lmin > GREP) {
    *over = true;
    return -1;
  }
  int depth = 0, p = q, a0 = 0;
  while (true) {
    if (++steps > GBUDGET) {
      *over = true;
      return -1;
    }
    int a = -1;
    for (int j = a0; j < nu; ++j)
      if (at(d, n, p, U[j].c, U[j].len)) {
        a = j;
        break;
      }
    if (a >= 0) {
      if (depth < lmin) {
        ch[depth] = (uint8_t)a;
        ps[depth] = p;
      }
      ++depth;
      p += U[a].len;
      a0 = 0;
      continue;
    }
    if (depth >= lmin) return p;  // stop here: the optional tail always matches
    if (depth == 0) return -1;
    --depth;
    p = ps[depth];
    a0 = ch[depth] + 1;
  }
}

// bits q .. q+63 of a match-table row (q >= 0; the padding words end every row)
GI uint64_t tb_at(const uint64_t* X, int nwt, int q) {
  const int w = q >> 6, o = q & 63;
  if (w >= nwt - 1) return 0ull;
  const uint64_t lo = X[w];
  return o ? (lo >> o) | (X[w + 1] << (64 - o)) : lo;
}

// The match tables of one (message, protocol) over the positions [base, n], lane = word: the unit and
// start occurrence bitmaps, then lmin rounds of
//   D_r = OR_a UA[a] & (D_{r-1} >> |U_a|),  D_0 = [base, n]
// -- the positions from which some sequence of r units matches.  sre's repetition below lmin backtracks
// over exactly these alternatives, so (?:U0|U1|..){lmin,} matches at q iff q is in D_lmin.  When one
// unit is a proper prefix of another (the only way two units match at one position, amb), the same
// rounds run over the first matching unit only (G_lmin: the greedy path reaches lmin units, so it is
// the path sre takes).  Returns 0 when D_lmin is empty, -1 when lmin exceeds the fallback's choice
// stack and the old step-by-step search would have tried a repetition (contract), else 1 with
// *succ = D_lmin, *gsucc = G_lmin (D_lmin when !amb).
GD int mu_tables(const Msg& m, int base, const Str* U, int nu, const Str& S, int lmin, bool amb,
                 const uint64_t** succ, const uint64_t** gsucc) {
  const int nwt = m.nwt, lane = lane_id();
  uint64_t* UA = m.tb;
  uint64_t* SA = UA + 3 * nwt;
  uint64_t* D[2] = {SA + nwt, SA + 2 * nwt};
  uint64_t* G[2] = {SA + 3 * nwt, SA + 4 * nwt};
  const int wb = base >> 6, we = m.n >> 6;
  const uint64_t lastm = (m.n & 63) == 63 ? ~0ull : (1ull << ((m.n & 63) + 1)) - 1;  // positions <= n
  uint64_t any = 0;
  for (int w = lane; w < nwt; w += 64) {
    const bool in = w >= wb && w <= we;
    uint64_t rng = in ? ~0ull : 0ull;
    if (w == wb) rng &= ~0ull << (base & 63);
    if (w == we) rng &= lastm;
    for (int a = 0; a < 3; ++a) {
      uint64_t acc = 0;
      if (a < nu && in) {
        acc = rng;
        for (int i = 0; i < U[a].len && acc; ++i) acc &= bm_at(m, U[a].c[i] - '0', w * 64 + i);
      }
      UA[a * nwt + w] = acc;
      any |= acc;
    }
    uint64_t sacc = 0;
    if (S.len && in) {
      sacc = rng;
      for (int i = 0; i < S.len && sacc; ++i) sacc &= bm_at(m, S.c[i] - '0', w * 64 + i);
    }
    SA[w] = sacc;
    D[0][w] = rng;
    D[1][w] = 0;
    G[0][w] = rng;
    G[1][w] = 0;
  }
  __syncthreads();  // (one wave per workgroup) the rows, LDS or global, are visible to every lane
  if (lmin > GREP && (S.len || ballot(any != 0))) return -1;
  int cur = 0;
  for (int r = 1; r <= lmin; ++r) {
    uint64_t nz = 0;
    for (int w = wb + lane; w <= we; w += 64) {
      uint64_t d = 0, g = 0, seen = 0;
      for (int a = 0; a < nu; ++a) {
        const uint64_t ua = UA[a * nwt + w];
        const int L = U[a].len;
        d |= ua & tb_at(D[cur], nwt, w * 64 + L);
        if (amb) {
          g |= ua & ~seen & tb_at(G[cur], nwt, w * 64 + L);
          seen |= ua;
        }
      }
      D[cur ^ 1][w] = d;
      if (amb) G[cur ^ 1][w] = g;
      nz |= d;
    }
    cur ^= 1;
    __syncthreads();
    if (!ballot(nz != 0)) return 0;  // no position starts r units: no match anywhere
  }
  *succ = D[cur];
  *gsucc = amb ? G[cur] : D[cur];
  return 1;
}

// first s >= from with the start string at s (every s without one) and s + |S| in succ, or -1:
// 64 words (4096 positions) per step, as find_bm
GD int find_ok(const Msg& m, int from, int slen, const uint64_t* succ) {
  const int nwt = m.nwt, we = m.n >> 6;
  const uint64_t* SA = m.tb + 3 * nwt;
  if (from < 0) from = 0;
  if (from > m.n) return -1;
  const int wf = from >> 6;
  for (int w0 = wf; w0 <= we; w0 += 64) {
    const int w = w0 + lane_id();
    uint64_t acc = 0;
    if (w <= we) {
      acc = tb_at(succ, nwt, w * 64 + slen);
      if (slen) acc &= SA[w];
      if (w == wf) acc &= ~0ull << (from & 63);
    }
    const uint64_t hit = ballot(acc != 0);
    if (hit) return bcast_i(acc ? w * 64 + ffs64(acc) : 0, ffs64(hit));
  }
  return -1;
}

// end of the greedy repetition from q: the first matching unit at every step until none matches.
// Units of one length L (the usual case) step 64 units per wave step (lane = unit).
GD int greedy_end(const Msg& m, const Str* U, int nu, int q) {
  const int nwt = m.nwt;
  const uint64_t* UA = m.tb;
  bool same = true;
  for (int a = 1; a < nu; ++a) same = same && U[a].len == U[0].len;
  if (same) {
    const int L = U[0].len;
    while (true) {
      const int p = q + lane_id() * L;
      bool hit = false;
      if (p <= m.n)
        for (int a = 0; a < nu; ++a) hit = hit || ((UA[a * nwt + (p >> 6)] >> (p & 63)) & 1ull);
      const uint64_t miss = ballot(!hit);
      if (miss) return q + ffs64(miss) * L;
      q += 64 * L;
    }
  }
  while (true) {
    int a = 0;
    for (; a < nu; ++a)
      if ((UA[a * nwt + (q >> 6)] >> (q & 63)) & 1ull) break;
    if (a == nu) return q;
    q += U[a].len;
  }
}

// any bit symbol 'F' (2) in b[0, n): 64 positions per step (wave-uniform callers)
GD bool any_f(const uint8_t* b, int n) {
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane_id();
    if (ballot(i < n && b[i] == 2)) return true;
  }
  return false;
}

// hex digits of bits b[0, nb) (helpers.py:28-64) into T; returns the count (after lstrip('0')).
// Lane = digit, 64 digits per step, compacted by ballot; T is read back by every lane afterwards
// (the barrier: T may be the slot's global scratch)
GD int hex_text(const uint8_t* b, int nb, int strip_zero, uint8_t* T) {
  const int nd = (nb + 3) >> 2, lane = lane_id();
  int q = 0;
  bool lead = strip_zero != 0;
  for (int d0 = 0; d0 < nd; d0 += 64) {
    const int d = d0 + lane;
    int v = 0;
    if (d < nd) {
      const int e = nb - 4 * (nd - 1 - d), a = (e - 4 > 0) ? e - 4 : 0;
      for (int i = a; i < e; ++i) v = (v << 1) | b[i];
    }
    bool keep = d < nd;
    if (lead) {  // leading zero digits are dropped up to the first non-zero one
      const uint64_t nz = ballot(d < nd && v != 0);
      if (!nz) continue;
      keep = keep && lane >= ffs64(nz);
      lead = false;
    }
    const uint64_t km = ballot(keep);
    if (keep) T[q + popc64(km & ((1ull << lane) - 1))] = (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10);
    q += popc64(km);
  }
  __syncthreads();  // one wave per workgroup: the digits of every lane are visible to all
  return q;
}

GD int emit(Sink& sk, const BankView& bv, int p, int pre_off, int pre_len, const uint8_t* T, int dl, int post_off,
            int post_len, int bitlen) {
  const int total = pre_len + dl + post_len;
  if (total > 65535) return SDX_RAISE_CONTRACT;  // sdx_result.payload_len
  if (sk.write) {  // the payload bytes spread over the wave, the record from lane 0
    uint8_t* dst = sk.heap + sk.hbase + sk.nheap;
    for (int i = lane_id(); i < total; i += 64)
      dst[i] = i < pre_len ? bv.str[pre_off + i] : i < pre_len + dl ? T[i - pre_len] : bv.str[post_off + i - pre_len - dl];
    if (lane_id() == 0) {
      sdx_result r;
      r.payload_off = sk.hbase + sk.nheap;
      r.payload_len = (uint16_t)total;
      r.proto = (uint16_t)p;
      r.bit_length = (uint32_t)bitlen;
      r.msg = sk.msg;
      sk.rec[sk.rbase + sk.nrec] = r;
    }
  }
  ++sk.nrec;
  sk.nheap += (uint32_t)total;
  return 0;
}

// ---------------------------------------------------------------------------------------------
// MU (message_unsynced.py:11-296)
// ---------------------------------------------------------------------------------------------
// one match's bits -> postDemodulation, padding, dmsg, modulematch, result (:226-290)
GD int finish_mu_g(const BankView& bv, const sdx_mu_proto* rec, int p, uint8_t* B, uint8_t* B2, uint8_t* T, int nb,
                   Sink& sk) {
  uint8_t* buf = B;
  if (rec->postdemo != SDX_PD_NONE && !any_f(buf, nb)) {  // 'F': int() ValueError caught -> unchanged
    int no = 0;
    const int rc = run_postdemo(rec->postdemo, buf, nb, B2, &no);
    if (rc == 0) return 0;  // rcode < 1
    if (rc == 1) {
      buf = B2;
      nb = no;
    }  // rc == -1: ValueError inside the method, caught -> bits unchanged
  }
  const int pad = rec->pad_bits;
  const int nbp = (nb + pad - 1) / pad * pad;  // (:257-259)
  for (int i = nb; i < nbp; ++i) buf[i] = 0;
  const bool isf = any_f(buf, nbp);
  int dl;
  if (rec->dispatch_bin) {  // (:264-265)
    for (int i = 0; i < nbp; ++i) T[i] = buf[i] == 2 ? 'F' : (uint8_t)('0' + buf[i]);
    dl = nbp;
  } else if (isf) {  // bin_str_2_hex_str -> None (helpers.py:44-45)
    if (rec->remove_zero) return SDX_RAISE_ATTRIBUTE;  // None.lstrip (:269)
    T[0] = 'N'; T[1] = 'o'; T[2] = 'n'; T[3] = 'e';  // f"{None}"
    dl = 4;
  } else {
    dl = hex_text(buf, nbp, rec->remove_zero, T);
  }
  if (rec->mm_dfa >= 0) {  // re.search(modulematch, payload) (:277-280); the preamble is in the state
    for (int i = 0; i < rec->post_len; ++i) T[dl + i] = bv.str[rec->post_off + i];
    if (!dfa_accepts(bv, rec->mm_dfa, rec->mm_pre_state, T, dl + rec->post_len)) return 0;
  }
  return emit(sk, bv, p, rec->pre_off, rec->pre_len, T, dl, rec->post_off, rec->post_len, nbp);
}

// protocols [p0, p1) of the bank (a chunk of the walk; chunks run in parallel, k_general_walk):
// returns the raise kind of the first protocol that raises (*raise_p = its index), else 0
GD int mu_chunk(const BankView& bv, Msg& m, int p0, int p1, uint8_t* B, uint8_t* B2, uint8_t* T, Sink& sk,
                int* raise_p) {
  if (m.n == 0) return 0;  // `if not raw_data` (:22-25)
  double last = __builtin_nan("");
  for (int p = p0; p < p1; ++p) {
    *raise_p = p;
    const sdx_mu_proto* rec = bv.mu + p;
    if (!rec->active || rec->never) continue;  // (:47-48); never = the key loop always fails
    if (!(rec->clock == last)) {
      last = rec->clock;
      for (int k = 0; k < m.npat; ++k) m.nv[k] = py_round1(m.val[k] / rec->clock);  // (:62-64)
    }
    int base = 0;
    Str& S = m.wk->str[0];
    S.len = 0;
    GP_T(tp0);
    if (rec->has_start) {  // (:70-88)
      const int r = pex(m, &rec->start, 0, &S);
      if (r < 0) return SDX_RAISE_CONTRACT;
      if (r == 0) continue;
      base = find_bm(m, 0, S);
    }
    // pattern_lookup (distinct strings, last writer), end_pattern_lookup (pstr[:-1], first writer)
    Str* U = m.wk->str + 1;
    Str* E = m.wk->str + 4;
    Str& t = m.wk->str[7];
    uint8_t* us = m.wk->sym;
    uint8_t* es = m.wk->sym + 3;
    int nu = 0, ne = 0;
    bool fail = false;
    const sdx_patspec* K[3] = {&rec->one, &rec->zero, &rec->flt};
    const uint8_t SYM[3] = {1, 0, 2};
    for (int k = 0; k < 3; ++k) {  // (:98-141)
      if (K[k]->len == 0) continue;
      const int r = pex(m, K[k], base, &t);
      if (r < 0) return SDX_RAISE_CONTRACT;
      if (r == 0) {
        if (k != 2) {
          fail = true;
          break;
        }
        continue;
      }
      int j = 0;
      for (; j < nu; ++j)
        if (str_eq(U[j], t, t.len)) break;
      if (j == nu) str_set(U[nu++], t, t.len);
      us[j] = SYM[k];
      if (t.len > 0) {
        int i = 0;
        for (; i < ne; ++i)
          if (str_eq(E[i], t, t.len - 1)) break;
        if (i == ne) {
          str_set(E[ne], t, t.len - 1);
          es[ne] = SYM[k];
          ++ne;
        }
      }
    }
    GP_ADD(0, tp0);
    if (fail || nu == 0) continue;
    GP_CNT(8);
    if (!rec->recon) ne = 0;  // the regex tail and the chunk fallback both need reconstructBit
    stage(m);
    const uint8_t* w = m.d + base;
    const int nw = m.n - base;
    const int W = rec->width;
    const int lmin = rec->length_min;
    bool amb = false;  // a unit that is a proper prefix of another: two units can match at one position
    for (int a = 0; a < nu; ++a)
      for (int b = 0; b < nu; ++b)
        if (U[a].len < U[b].len && str_eq(U[a], U[b], U[a].len)) amb = true;
    GP_T(tt0);
    const uint64_t *succ = nullptr, *gsucc = nullptr;
    const int tr = mu_tables(m, base, U, nu, S, lmin, amb, &succ, &gsucc);
    GP_ADD(11, tt0);
    if (tr < 0) return SDX_RAISE_CONTRACT;
    if (tr == 0) continue;
    int pos = 0;
    while (pos <= nw) {  // matcher.finditer(current_raw_data) (:195)
      GP_T(tf0);
      const int sa = find_ok(m, base + pos, S.len, succ);  // the leftmost position the regex matches at
      GP_ADD(1, tf0);
      if (sa < 0) break;
      const int s = sa - base, gq = s + S.len;
      int ge;
      GP_T(tr0);
      if ((gsucc[(sa + S.len) >> 6] >> ((sa + S.len) & 63)) & 1ull) {
        ge = greedy_end(m, U, nu, sa + S.len) - base;
      } else {  // below lmin the greedy path dead-ends: sre's backtracking order, step by step
        bool over = false;
        ge = rep_match(w, nw, gq, U, nu, lmin, &over, m.wk->ch, m.wk->ps);
        GP_CNT(12);
        if (over) return SDX_RAISE_CONTRACT;
        if (ge < 0) {  // unreachable: gq is in D_lmin
          pos = s + 1;
          continue;
        }
      }
      GP_ADD(2, tr0);
      for (int j = 0; j < ne; ++j)  // (?:E0|E1|..)? : the first key that matches
        if (at(w, nw, ge, E[j].c, E[j].len)) {
          ge += E[j].len;
          break;
        }
      pos = ge > s ? ge : s + 1;
      if (W == 0) continue;  // (:204-205)
      const int glen = ge - gq;
      if (glen == 0) return SDX_RAISE_INDEX;  // chunks[-1] on [] (:212)
      const int nch = (glen + W - 1) / W;
      if (nch > rec->length_max) continue;  // (:217-218); INT32_MAX = no length_max
      GP_CNT(10);
      GP_T(tc0);
      int nb = 0;
      for (int c0 = 0; c0 < nch; c0 += 64) {  // (:220-229), lane = chunk; unmatched chunks are skipped
        const int c = c0 + lane_id();
        int sy = -1;
        if (c < nch) {
          const int x = gq + c * W, cl = (ge - x < W) ? ge - x : W;
          for (int j = 0; j < nu && sy < 0; ++j)
            if (U[j].len == cl && at(w, nw, x, U[j].c, cl)) sy = us[j];
          for (int j = 0; j < ne && sy < 0; ++j)
            if (E[j].len == cl && at(w, nw, x, E[j].c, cl)) sy = es[j];
        }
        const uint64_t hit = ballot(sy >= 0);
        if (sy >= 0) B[nb + popc64(hit & ((1ull << lane_id()) - 1))] = (uint8_t)sy;
        nb += popc64(hit);
      }
      __syncthreads();  // B (the slot's global scratch) is read by every lane from here on
      GP_ADD(3, tc0);
      GP_T(tz0);
      const int rr = finish_mu_g(bv, rec, p, B, B2, T, nb, sk);
      GP_ADD(4, tz0);
      if (rr) return rr;
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// MS (message_synced.py:10-243)
// ---------------------------------------------------------------------------------------------
GD int finish_ms_g(const BankView& bv, const sdx_ms_proto* rec, int p, uint8_t* B, uint8_t* B2, uint8_t* T, int nb,
                   Sink& sk) {
  uint8_t* buf = B;
  if (nb == 0) return 0;                                           // (:191-192)
  if (rec->lir_min != -1 && nb < rec->lir_min) return 0;           // length_in_range (:194-196)
  if (nb > rec->lir_max) return 0;
  const int pad = rec->pad_bits;                                   // padding before postDemod (:198-200)
  const int nbp = (nb + pad - 1) / pad * pad;
  for (int i = nb; i < nbp; ++i) buf[i] = 0;
  nb = nbp;
  if (rec->postdemo != SDX_PD_NONE) {                             // no try: 'F' raises ValueError (:209)
    if (any_f(buf, nb)) return SDX_RAISE_VALUE;
    int no = 0;
    const int rc = run_postdemo(rec->postdemo, buf, nb, B2, &no);
    if (rc == -1) return SDX_RAISE_VALUE;
    if (rc == 0) return 0;
    if (no > 0) {  // `if ret_bits`
      buf = B2;
      nb = no;
    }
  }
  if (any_f(buf, nb)) return 0;  // bin_str_2_hex_str -> None -> skipped (:224-226)
  const int dl = hex_text(buf, nb, 0, T);
  return emit(sk, bv, p, rec->pre_off, rec->pre_len, T, dl, rec->post_off, rec->post_len, nb);
}

GD int ms_chunk(const BankView& bv, Msg& m, int cp, bool ok, int p0, int p1, uint8_t* B, uint8_t* B2, uint8_t* T,
                Sink& sk, int* raise_p) {
  if (!ok || cp < 0 || cp >= m.npat) return 0;  // the string gates and `str(CP) in patterns` (:21-57)
  const double clock = fabs(m.val[cp]);
  if (clock == 0.0) return 0;  // (:60-62)
  for (int k = 0; k < m.npat; ++k) m.nv[k] = py_round1(m.val[k] / clock);  // (:64-72)
  const uint8_t KS[4] = {3, 1, 0, 2};  // sync '', one '1', zero '0', float 'F'
  for (int p = p0; p < p1; ++p) {
    *raise_p = p;
    const sdx_ms_proto* rec = bv.ms + p;
    if (rec->never) continue;
    if (rec->pclock > 0.0 && fabs(rec->pclock - clock) > clock * 0.3) continue;  // (:81-86)
    const int W = rec->width;
    Str* K = m.wk->str;
    Str* E = m.wk->str + 4;
    Str& t = m.wk->str[7];
    uint8_t* ks = m.wk->sym;
    uint8_t* es = m.wk->sym + 4;
    int nk = 0, ne = 0, mstart = 0;
    bool fail = false;
    for (int k = 0; k < 4; ++k) {  // (:109-160)
      const sdx_patspec* sp = &rec->key[k];
      if (sp->len == 0) continue;
      const int r = pex(m, sp, 0, &t);
      if (r < 0) return SDX_RAISE_CONTRACT;
      if (r == 0) {
        if (k != 3) {
          fail = true;
          break;
        }
        continue;
      }
      int j = 0;
      for (; j < nk; ++j)
        if (str_eq(K[j], t, t.len)) break;
      if (j == nk) str_set(K[nk++], t, t.len);
      ks[j] = KS[k];
      if (t.len > 0) {
        int i = 0;
        for (; i < ne; ++i)
          if (str_eq(E[i], t, t.len - 1)) break;
        if (i == ne) {
          str_set(E[ne], t, t.len - 1);
          es[ne] = KS[k];
          ++ne;
        }
      }
      if (k == 0) {  // (:145-158)
        mstart = find_bm(m, 0, t) + t.len;
        const double bl = W > 0 ? (double)(m.n - mstart) / (double)W : 0.0;
        if ((double)rec->lmin_sync > bl) {
          fail = true;
          break;
        }
        ne = 0;  // end_pattern_lookup = {}
      }
    }
    if (fail || nk == 0 || W <= 0) continue;
    stage(m);
    int nb = 0;
    for (int i = mstart; i < m.n; i += W) {  // (:172-189)
      const int cl = (m.n - i < W) ? m.n - i : W;
      int sy = -1;
      for (int j = 0; j < nk && sy < 0; ++j)
        if (K[j].len == cl && at(m.d, m.n, i, K[j].c, cl)) sy = ks[j];
      if (sy >= 0) {
        if (sy != 3) B[nb++] = (uint8_t)sy;
        continue;
      }
      if (!rec->recon) break;
      const int tl = cl == W ? cl - 1 : cl;  // chunk[:-1] if full else chunk
      for (int j = 0; j < ne && sy < 0; ++j)
        if (E[j].len == tl && at(m.d, m.n, i, E[j].c, tl)) sy = es[j];
      if (sy < 0) break;
      B[nb++] = (uint8_t)sy;
    }
    const int rr = finish_ms_g(bv, rec, p, B, B2, T, nb, sk);
    if (rr) return rr;
  }
  return 0;
}

// Work split: the bank walk of a message is cut into chunks of GCH protocols, and a (message, chunk)
// item is one wave's work.  A persistent grid of waves takes items from a device counter (heaviest
// messages first: the host orders them by length), every lane of a wave running the same serial
// walk on the same state (all control flow wave-uniform) with the wide steps -- str.find over the
// character bitmaps, payload copies -- spread over the 64 lanes.  A message's results and raise are
// the concatenation of its chunks in bank order up to the first raising protocol (message_unsynced.py
// :45-49: an exception leaves the protocol loop), so:
//   k_gen_prep     wave per message: its digit-character bitmaps into its workspace region;
//   k_gen_walk<0>  every item: count its chunk's results and payload bytes, note the first raise;
//   k_gen_reserve  thread per message: first raise over its chunks in bank order, else one
//                  record / heap reservation for the message and each chunk's base;
//   k_gen_walk<1>  items with results of messages that did not raise: the same walk, writing.
constexpr int GCH = 1;          // protocols per chunk (one: the most parallel; staging a message costs ~us)
constexpr int GSLOTS = 1024;    // resident waves of the walk (scratch slots)
constexpr int GHEAD = (int)((sizeof(Msg) + sizeof(Wk) + 15) & ~(size_t)15);  // LDS: Msg, Wk, then data
__host__ __device__ inline int lds_need(int n) { return GHEAD + ((n + 7) & ~7); }                   // + the message's characters
__host__ __device__ inline int64_t lds_need_tb(int n) { return lds_need(n) + tb_bytes(n); }             // + the match tables
// per-slot scratch: bits, postDemod output and payload text (max_len + GSLACK bytes each), then the
// match tables of a message whose tables do not fit the LDS
__host__ __device__ inline int64_t slot_bytes(int max_len) {
  return ((3 * ((int64_t)max_len + GSLACK) + 255) & ~(int64_t)255) + ((tb_bytes(max_len) + 255) & ~(int64_t)255);
}

struct GenChunk {  // per (message, chunk); 24 bytes
  uint32_t nrec, nheap, rbase, hbase;
  uint32_t raise;  // raise kind << 16 | protocol (0: none)
  uint32_t res;
};

// workspace: [item counters (256 B) | chunk table | slot scratch | per-message regions]
struct GenPlan {
  int64_t tab, head;  // byte offsets of the slot scratch and of the per-message regions
  int nproto, nch, max_len, slots, lds;
};

// the per-message region: the message's bitmaps (k_gen_prep)
GI uint8_t* gen_region(const sdx_general_batch& b, const sdx_out& out, const GenPlan& g, int i, int msg) {
  return out.work_dev + g.head +
         (b.work_stride > 0 ? (int64_t)i * b.work_stride : 5 * b.offsets_dev[msg] + (int64_t)5 * GSLACK * msg);
}
GI uint32_t* gen_ctr(const sdx_out& out) { return reinterpret_cast<uint32_t*>(out.work_dev); }
GI GenChunk* gen_table(const sdx_out& out) { return reinterpret_cast<GenChunk*>(out.work_dev + 256); }
GI uint8_t* gen_slot(const sdx_out& out, const GenPlan& g, int slot) {
  return out.work_dev + g.tab + (int64_t)slot * slot_bytes(g.max_len);
}

__global__ __launch_bounds__(64) void k_gen_prep(sdx_general_batch b, sdx_out out, GenPlan g) {
  const int i = blockIdx.x, lane = threadIdx.x;
  const int msg = b.sel_dev ? b.sel_dev[i] : i;
  const int64_t off = b.offsets_dev[msg];
  const uint8_t* d = b.data_dev + off;
  const int n = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - off);
  if (n > g.max_len) return;  // outside the batch's max_len: k_gen_walk raises SDX_RAISE_CONTRACT for it
  const int nwp = ((n + 63) >> 6) + 1;
  uint64_t* bmw = reinterpret_cast<uint64_t*>(gen_region(b, out, g, i, msg));
  if (i == 0 && lane < 2) gen_ctr(out)[lane] = 0;  // the two walk passes' item counters
  for (int w = lane; w < nwp; w += 64) {  // lane l builds words l, l + 64, ..
    uint64_t a[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) a[c] = 0;
    const int p0 = w * 64, pe = (n - p0 < 64) ? n - p0 : 64;
    for (int j = 0; j < pe; ++j) {
      const int c = (int)d[p0 + j] - '0';
#pragma unroll
      for (int k = 0; k < 10; ++k) a[k] |= (uint64_t)(c == k) << j;
    }
#pragma unroll
    for (int c = 0; c < 10; ++c) bmw[(size_t)c * nwp + w] = a[c];
  }
}

template <int KIND, int PASS>
__global__ __launch_bounds__(64) void k_gen_walk(const void* __restrict__ bank, sdx_general_batch b, sdx_out out,
                                                 GenPlan g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t glds[];
  const BankView bv = bank_view(bank);
  const int lane = threadIdx.x;
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const int nitems = ntot * g.nch;
  uint32_t* ctr = gen_ctr(out) + PASS;
  GenChunk* tab = gen_table(out);
  // per-slot scratch: bits, postDemod output, payload text (every lane writes the same bytes and reads
  // back only what it wrote itself)
  uint8_t* B = gen_slot(out, g, blockIdx.x);
  uint8_t* B2 = B + g.max_len + GSLACK;
  uint8_t* T = B2 + g.max_len + GSLACK;
  uint64_t* TBG = reinterpret_cast<uint64_t*>(B + ((3 * ((int64_t)g.max_len + GSLACK) + 255) & ~(int64_t)255));
  Msg& m = *reinterpret_cast<Msg*>(glds);
  m.wk = reinterpret_cast<Wk*>(glds + sizeof(Msg));
  int cur = -1;  // the item's message whose characters / bitmaps are staged
  while (true) {
    int item = 0;
    if (lane == 0) item = (int)atomicAdd(ctr, 1u);
    item = bcast_i(item, 0);
    if (item >= nitems) break;
    const int i = item / g.nch, c = item - i * g.nch;
    const int msg = b.sel_dev ? b.sel_dev[i] : i;
    GenChunk& e = tab[item];
    if (PASS == 1 && (e.nrec == 0 || out.desc_dev[msg].status != SDX_ST_OK)) continue;
    const int p0 = c * GCH, p1 = (p0 + GCH < g.nproto) ? p0 + GCH : g.nproto;
    if (GCH == 1 && PASS == 0) {  // a protocol the walk skips anyway: no staging
      const bool skip = KIND == SDX_KIND_MU ? (!bv.mu[p0].active || bv.mu[p0].never) : (bool)bv.ms[p0].never;
      if (skip) {
        if (lane == 0) {
          e.nrec = 0;
          e.nheap = 0;
          e.raise = 0;
        }
        continue;
      }
    }
    GP_T(ti0);
    if (i != cur) {  // stage the message (the LDS holds one)
      cur = i;
      const int64_t off = b.offsets_dev[msg];
      m.d = b.data_dev + off;
      m.n = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - off);
      m.npat = b.npat_dev[msg] < GP ? b.npat_dev[msg] : GP;
      m.ids = b.pat_ids_dev + (size_t)msg * GP * GID;
      m.val = b.pat_val_dev + (size_t)msg * GP;
      m.nwp = ((m.n + 63) >> 6) + 1;
      const uint64_t* gbm = reinterpret_cast<const uint64_t*>(gen_region(b, out, g, i, msg));
      m.bm = gbm;  // the digit bitmaps are read by the wide steps only (64 lanes): they stay in HBM / L2
      m.nwt = tb_words(m.n);
      m.tb = TBG;
      m.ld = nullptr;
      m.staged = 0;
      if (lds_need(m.n) <= g.lds) {  // the characters (stage()) and the match tables at LDS latency
        m.ld = glds + GHEAD;
        if (lds_need_tb(m.n) <= g.lds) m.tb = reinterpret_cast<uint64_t*>(glds + lds_need(m.n));
      }
    }
    GP_ADD(5, ti0);
    if (m.n > g.max_len) {  // the per-slot scratch and regions are sized by max_len: never walk past them
      if (PASS == 0 && lane == 0) {
        e.nrec = 0;
        e.nheap = 0;
        e.raise = ((uint32_t)SDX_RAISE_CONTRACT << 16) | (uint32_t)p0;
      }
      continue;
    }
    Sink sk{PASS == 1, 0, 0u, out.rec_dev, out.heap_dev, PASS == 1 ? e.rbase : 0u, PASS == 1 ? e.hbase : 0u,
            (uint32_t)msg};
    int rp = 0, raise;
    if (KIND == SDX_KIND_MU) {
      raise = mu_chunk(bv, m, p0, p1, B, B2, T, sk, &rp);
    } else {
      const int cp = (int)b.cp_slot_dev[msg];
      raise = ms_chunk(bv, m, cp, b.ms_ok_dev[msg] != 0, p0, p1, B, B2, T, sk, &rp);
    }
    if (PASS == 0 && lane == 0) {
      e.nrec = (uint32_t)sk.nrec;
      e.nheap = sk.nheap;
      e.raise = raise ? ((uint32_t)raise << 16) | (uint32_t)rp : 0u;
#ifdef SDX_GPROF
      e.res = (uint32_t)(__builtin_amdgcn_s_memtime() - ti0);
#endif
    }
    GP_ADD(6 + PASS, ti0);
  }
}

// thread per message: its chunks in bank order -> the first raise, or one reservation and the chunk bases
__global__ __launch_bounds__(256) void k_gen_reserve(sdx_general_batch b, sdx_out out, GenPlan g) {
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= ntot) return;
  const int msg = b.sel_dev ? b.sel_dev[i] : i;
  GenChunk* e = gen_table(out) + (int64_t)i * g.nch;
  sdx_desc d;
  d.rec_begin = 0;
  d.n_rec = 0;
  d.status = SDX_ST_OK;
  d.raise_kind = 0;
  uint64_t nr = 0, nh = 0;
  for (int c = 0; c < g.nch; ++c) {
    if (e[c].raise) {
      d.status = SDX_ST_RAISED;
      d.raise_kind = (uint8_t)(e[c].raise >> 16);
      break;
    }
    nr += e[c].nrec;
    nh += e[c].nheap;
  }
  if (d.status == SDX_ST_OK && nr) {
    const uint32_t nh16 = (uint32_t)((nh + 15) & ~15ull);
    const uint32_t rb = atomicAdd(&out.cursor_dev[0], (uint32_t)nr);
    const uint32_t hb = atomicAdd(&out.cursor_dev[1], nh16);
    if (nr > 65535 || nh > 0xFFFFFFF0ull || (uint64_t)rb + nr > out.rec_cap || (uint64_t)hb + nh16 > out.heap_cap) {
      d.status = SDX_ST_OVF_OUT;
      atomicOr(&out.cursor_dev[2], 1u);
    } else {
      uint32_t r = rb, h = hb;
      for (int c = 0; c < g.nch; ++c) {
        e[c].rbase = r;
        e[c].hbase = h;
        r += e[c].nrec;
        h += e[c].nheap;
      }
      d.rec_begin = rb;
      d.n_rec = (uint16_t)nr;
    }
  }
  out.desc_dev[msg] = d;
}

// ---------------------------------------------------------------------------------------------
// MC frames of any length: the "fixed" chain of k_mc (manchester.py:49-144) with the frame's bits
// in global memory (LaneBits layout: word w of lane t at base[w * 256 + t])
// ---------------------------------------------------------------------------------------------
GD int mc_frame(const BankView& bv, const LaneBits& BN, const LaneBits& BI, int nN, int nI, bool hex_ok, int clock,
                int mcbit, int flags, int mw, int only, Sink& sk) {
  const int nmc = (int)bv.hdr->n_mc;
  for (int p = 0; p < nmc; ++p) {
    if (only >= 0 && p != only) continue;
    const sdx_mc_proto* r = bv.mc + p;
    // gates of _demodulate_mc_data (manchester.py:70-89; clockrange fixed to [0] / [1])
    if (mcbit < (r->has_lmin ? r->lmin : -1)) continue;
    if (mcbit > (r->has_lmax ? r->lmax : 9999)) continue;
    if (r->has_cr && !((double)clock > r->cr_lo && (double)clock < r->cr_hi)) continue;
    if (!hex_ok) return SDX_RAISE_TYPE;  // len(None) -> TypeError
    const bool inv = (r->invert != 0) ^ ((flags & 3) != 0);  // (:91-96)
    const LaneBits& B = inv ? BI : BN;
    const int nb = inv ? nI : nN;
    const LaneBits DM{B.base, mw, true};
    const McOut o = mc_method(r, r->method, B, nb, nb, DM);
    if (o.rc == -1) return SDX_RAISE_TYPE;
    if (o.rc == -2) return SDX_RAISE_VALUE;
    if (o.rc != 1) continue;
    const int total = r->pre_len + o.len;
    if (total > 65535) return SDX_RAISE_CONTRACT;
    if (sk.write) {
      uint8_t* dst = sk.heap + sk.hbase + sk.nheap;
      for (int i = 0; i < r->pre_len; ++i) dst[i] = bv.str[r->pre_off + i];
      mc_write(r, o, B, nb, nb, dst + r->pre_len);
      sdx_result x;
      x.payload_off = sk.hbase + sk.nheap;
      x.payload_len = (uint16_t)total;
      x.proto = (uint16_t)p;
      x.bit_length = 0;
      x.msg = sk.msg;
      sk.rec[sk.rbase + sk.nrec] = x;
    }
    ++sk.nrec;
    sk.nheap += (uint32_t)total;
  }
  return 0;
}

__global__ __launch_bounds__(256) void k_mc_general(const void* __restrict__ bank, sdx_mc_batch b, int mw, sdx_out out) {
  const BankView bv = bank_view(bank);
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const int tid = threadIdx.x, gi = blockIdx.x * 256 + tid;
  if (gi >= ntot) return;
  const int msg = b.sel_dev ? b.sel_dev[gi] : gi;
  uint64_t* bn = reinterpret_cast<uint64_t*>(out.work_dev) + (size_t)blockIdx.x * 512 * mw + tid;
  uint64_t* bi = bn + (size_t)256 * mw;
  const int64_t off = b.offsets_dev[msg];
  const int hl = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - off);
  // hex -> bits of both polarities (helpers.py:168-188: leading zero nibbles dropped; the
  // _convert_mc_hex_to_bits translate inverts uppercase digits only, manchester.py:33-36)
  bool hex_ok = hl > 0 && hl <= mw * 16;
  int nN = 0, nI = 0;
  bool startedN = false, startedI = false;
  uint64_t wn = 0, wi = 0;
  for (int i = 0; i < hl && hex_ok; ++i) {
    const uint8_t c = b.hex_dev[off + i];
    int v = -1;
    if (c >= '0' && c <= '9') v = c - '0';
    else if (c >= 'A' && c <= 'F') v = c - 'A' + 10;
    else if (c >= 'a' && c <= 'f') v = c - 'a' + 10;
    if (v < 0) {
      hex_ok = false;
      break;
    }
    const bool upper = !(c >= 'a' && c <= 'f');
    const int vi = upper ? 15 - v : v;
    if (v || startedN || i == hl - 1) {
      startedN = true;
      wn |= (uint64_t)v << (60 - (nN & 63));
      nN += 4;
      if ((nN & 63) == 0) { bn[(size_t)((nN >> 6) - 1) * 256] = wn; wn = 0; }
    }
    if (vi || startedI || i == hl - 1) {
      startedI = true;
      wi |= (uint64_t)vi << (60 - (nI & 63));
      nI += 4;
      if ((nI & 63) == 0) { bi[(size_t)((nI >> 6) - 1) * 256] = wi; wi = 0; }
    }
  }
  if (!hex_ok) {  // no method runs on these bits (TypeError before any decode)
    nN = nI = 0;
    wn = wi = 0;
  }
  for (int w = nN >> 6; w < mw; ++w) { bn[(size_t)w * 256] = (w == (nN >> 6)) ? wn : 0ull; }
  for (int w = nI >> 6; w < mw; ++w) { bi[(size_t)w * 256] = (w == (nI >> 6)) ? wi : 0ull; }
  const LaneBits BN{bn, mw, false}, BI{bi, mw, false};
  const int clock = b.clock_dev[msg], mcbit = b.mcbitnum_dev[msg], flags = b.flags_dev[msg];
  const int only = b.only_dev ? b.only_dev[msg] : -1;
  Sink sk{false, 0, 0u, out.rec_dev, out.heap_dev, 0u, 0u, (uint32_t)msg};
  int raise = mc_frame(bv, BN, BI, nN, nI, hex_ok, clock, mcbit, flags, mw, only, sk);
  sdx_desc d;
  d.rec_begin = 0;
  d.n_rec = 0;
  d.raise_kind = (uint8_t)raise;
  d.status = raise ? SDX_ST_RAISED : SDX_ST_OK;
  if (!raise && sk.nrec) {
    const uint32_t nh = (sk.nheap + 15u) & ~15u;
    const uint32_t rb = atomicAdd(&out.cursor_dev[0], (uint32_t)sk.nrec);
    const uint32_t hb = atomicAdd(&out.cursor_dev[1], nh);
    if (rb + sk.nrec > out.rec_cap || hb + nh > out.heap_cap) {
      d.status = SDX_ST_OVF_OUT;
      atomicOr(&out.cursor_dev[2], 1u);
    } else {
      Sink sw{true, 0, 0u, out.rec_dev, out.heap_dev, rb, hb, (uint32_t)msg};
      mc_frame(bv, BN, BI, nN, nI, hex_ok, clock, mcbit, flags, mw, only, sw);
      d.rec_begin = rb;
      d.n_rec = (uint16_t)sw.nrec;
    }
  }
  out.desc_dev[msg] = d;
}

}  // namespace sdxg

extern "C" {

#ifdef SDX_GPROF
int sdx_genprof_read(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(sdxg::g_genprof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(sdxg::g_genprof), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

static sdxg::GenPlan gen_plan(const sdx_bank* bank, int kind, int32_t n, int32_t max_len) {
  sdxg::GenPlan g;
  const sdx_bank_hdr* h = sdx::bank_hdr(bank);
  g.nproto = kind == SDX_KIND_MU ? (int)h->n_mu : (int)h->n_ms;
  g.nch = (g.nproto + sdxg::GCH - 1) / sdxg::GCH;
  if (g.nch < 1) g.nch = 1;
  g.max_len = max_len > 0 ? max_len : 0;
  const int64_t items = (int64_t)(n > 0 ? n : 0) * g.nch;
  g.slots = (int)(items < sdxg::GSLOTS ? (items > 0 ? items : 1) : sdxg::GSLOTS);
  g.tab = 256 + (((int64_t)(n > 0 ? n : 0) * g.nch * (int64_t)sizeof(sdxg::GenChunk) + 255) & ~(int64_t)255);
  g.head = g.tab + (int64_t)g.slots * sdxg::slot_bytes(g.max_len);
  // LDS per wave: the working set plus the longest message's characters and match tables, at most
  // 64 KB (what does not fit stays in HBM: the tables first)
  const int64_t ntb = sdxg::lds_need_tb(g.max_len);
  g.lds = ntb <= 65536 ? (int)ntb : (sdxg::lds_need(g.max_len) <= 65536 ? sdxg::lds_need(g.max_len) : sdxg::GHEAD);
  return g;
}

uint64_t sdx_general_work_bytes(const sdx_bank* bank, int kind, int64_t total_chars, int32_t n, int32_t max_len,
                                int64_t work_stride) {
  if (!bank || (kind != SDX_KIND_MU && kind != SDX_KIND_MS)) return 0;
  const sdxg::GenPlan g = gen_plan(bank, kind, n, max_len);
  const int64_t regions = work_stride > 0 ? work_stride * (int64_t)(n > 0 ? n : 0)
                                          : 5 * (total_chars > 0 ? total_chars : 0) +
                                                (int64_t)5 * sdxg::GSLACK * (n > 0 ? n : 0);
  return (uint64_t)(g.head + regions + 256);
}

int sdx_demod_pulses_general(const sdx_bank* bank, int kind, const sdx_general_batch* batch, const sdx_out* out,
                             void* hip_stream) {
  if (!bank || !batch || !out) return sdx::set_error(SDX_EINVAL, "null argument");
  if (kind != SDX_KIND_MU && kind != SDX_KIND_MS) return sdx::set_error(SDX_EINVAL, "kind must be MU or MS");
  if (kind == SDX_KIND_MS && (!batch->cp_slot_dev || !batch->ms_ok_dev))
    return sdx::set_error(SDX_EINVAL, "MS needs cp_slot/ms_ok");
  const int ntot = batch->sel_dev ? batch->n_sel : batch->n;
  if (ntot <= 0) return SDX_OK;
  if (!batch->data_dev || !batch->offsets_dev || !batch->npat_dev || !batch->pat_ids_dev || !batch->pat_val_dev ||
      !out->work_dev || batch->max_len < 0)
    return sdx::set_error(SDX_EINVAL, "sdx_demod_pulses_general: missing buffer");
  if (batch->work_stride > 0 && batch->work_stride < 5 * ((int64_t)batch->max_len + sdxg::GSLACK))
    return sdx::set_error(SDX_EINVAL, "sdx_demod_pulses_general: work_stride < 5 * (max_len + 512)");
  // the regions' part of the workspace is the caller's (sdx_general_work_bytes); the head is checked here
  const sdxg::GenPlan g = gen_plan(bank, kind, ntot, batch->max_len);
  if (out->work_cap < (uint64_t)g.head) return sdx::set_error(SDX_EINVAL, "sdx_demod_pulses_general: work_cap < sdx_general_work_bytes");
  hipStream_t st = (hipStream_t)hip_stream;
  const void* bd = sdx::bank_dev_ptr(bank);
  const int nitems = ntot * g.nch;
  const int grid = nitems < g.slots ? nitems : g.slots;
  hipLaunchKernelGGL(sdxg::k_gen_prep, dim3(ntot), dim3(64), 0, st, *batch, *out, g);
  if (kind == SDX_KIND_MU)
    hipLaunchKernelGGL((sdxg::k_gen_walk<SDX_KIND_MU, 0>), dim3(grid), dim3(64), g.lds, st, bd, *batch, *out, g);
  else
    hipLaunchKernelGGL((sdxg::k_gen_walk<SDX_KIND_MS, 0>), dim3(grid), dim3(64), g.lds, st, bd, *batch, *out, g);
  hipLaunchKernelGGL(sdxg::k_gen_reserve, dim3((ntot + 255) / 256), dim3(256), 0, st, *batch, *out, g);
  if (kind == SDX_KIND_MU)
    hipLaunchKernelGGL((sdxg::k_gen_walk<SDX_KIND_MU, 1>), dim3(grid), dim3(64), g.lds, st, bd, *batch, *out, g);
  else
    hipLaunchKernelGGL((sdxg::k_gen_walk<SDX_KIND_MS, 1>), dim3(grid), dim3(64), g.lds, st, bd, *batch, *out, g);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("k_gen_*: ") + hipGetErrorString(e));
  return SDX_OK;
}

uint64_t sdx_mc_general_work_bytes(int32_t n, int32_t max_hex) {
  const int64_t mw = ((int64_t)(max_hex > 0 ? max_hex : 1) + 15) / 16;
  const int64_t blocks = ((int64_t)(n > 0 ? n : 0) + 255) / 256;
  return (uint64_t)(blocks * 512 * mw * 8);
}

int sdx_demod_mc_general(const sdx_bank* bank, const sdx_mc_batch* batch, int32_t max_hex, const sdx_out* out,
                         void* hip_stream) {
  if (!bank || !batch || !out) return sdx::set_error(SDX_EINVAL, "null argument");
  const int ntot = batch->sel_dev ? batch->n_sel : batch->n;
  if (ntot <= 0) return SDX_OK;
  if (max_hex <= 0 || !out->work_dev || out->work_cap < sdx_mc_general_work_bytes(ntot, max_hex))
    return sdx::set_error(SDX_EINVAL, "sdx_demod_mc_general: work_dev smaller than sdx_mc_general_work_bytes");
  const int mw = (max_hex + 15) / 16;
  hipLaunchKernelGGL(sdxg::k_mc_general, dim3((ntot + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream,
                     sdx::bank_dev_ptr(bank), *batch, mw, *out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("k_mc_general: ") + hipGetErrorString(e));
  return SDX_OK;
}

}  // extern "C"
