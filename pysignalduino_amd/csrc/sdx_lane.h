// sdx_lane.h -- lane-per-message primitives for messages of <= 64*NW pulses (NW <= 4).
//
// A message's position bitmaps live in LDS (one u64 word per 64 pulses per pattern id); here
// every mask that one (message x protocol) pair needs -- a target's occurrences, the unit
// positions, "a run of >= m units starts here" -- is an NW-word register array, so a wave runs
// 64 independent messages through pattern_exists AND through the exact re.finditer emulation
// without any cross-lane traffic.  Bit p of the mask = position p of the message.
#pragma once
#include "sdx_device.h"

namespace sdx {

template <int NW>
struct M {
  uint64_t w[NW];
};

template <int NW>
SDX_DEV M<NW> m_all() {
  M<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = ~0ull;
  return r;
}
template <int NW>
SDX_DEV M<NW> m_zero() {
  M<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = 0ull;
  return r;
}
template <int NW>
SDX_DEV M<NW> m_and(const M<NW>& a, const M<NW>& b) {
  M<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] & b.w[i];
  return r;
}
template <int NW>
SDX_DEV M<NW> m_or(const M<NW>& a, const M<NW>& b) {
  M<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] | b.w[i];
  return r;
}
template <int NW>
SDX_DEV M<NW> m_not(const M<NW>& a) {
  M<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = ~a.w[i];
  return r;
}
// word i of a, selected with bit masks (no dynamic register indexing -> no scratch)
template <int NW>
SDX_DEV uint64_t m_word(const M<NW>& a, int i) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) v |= a.w[k] & (0ull - (uint64_t)(i == k));
  return v;
}
// out bit p = a bit (p + r), 0 <= r < 64 (no dynamic word indexing)
template <int NW>
SDX_DEV M<NW> m_shr_small(const M<NW>& a, int r) {
  M<NW> o;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint64_t hi = (i + 1 < NW) ? a.w[i + 1] : 0ull;
    o.w[i] = r ? ((a.w[i] >> r) | (hi << (64 - r))) : a.w[i];
  }
  return o;
}
// out bit p = a bit (p - r), 0 <= r < 64
template <int NW>
SDX_DEV M<NW> m_shl_small(const M<NW>& a, int r) {
  M<NW> o;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint64_t lo = (i > 0) ? a.w[i - 1] : 0ull;
    o.w[i] = r ? ((a.w[i] << r) | (lo >> (64 - r))) : a.w[i];
  }
  return o;
}
// out bit p = a bit (p + s): positions move DOWN by s (s >= 0)
template <int NW>
SDX_DEV M<NW> m_shr(const M<NW>& a, int s) {
  const int q = s >> 6;
  if (q == 0) return m_shr_small(a, s);
  M<NW> b;
#pragma unroll
  for (int i = 0; i < NW; ++i) b.w[i] = m_word(a, i + q);
  return m_shr_small(b, s & 63);
}
// reverse the 4 bits inside every nibble (packed-LSB-first bits -> hex digit values)
SDX_DEV uint64_t nibrev(uint64_t x) {
  x = ((x & 0x5555555555555555ull) << 1) | ((x >> 1) & 0x5555555555555555ull);
  x = ((x & 0x3333333333333333ull) << 2) | ((x >> 2) & 0x3333333333333333ull);
  return x;
}
// first set bit at position >= from, or -1
template <int NW>
SDX_DEV int m_first(const M<NW>& a, int from) {
  int res = -1;
#pragma unroll
  for (int i = NW - 1; i >= 0; --i) {
    uint64_t x = a.w[i];
    const int lo = from - 64 * i;
    if (lo >= 64) x = 0;
    else if (lo > 0) x &= ~0ull << lo;
    if (x) res = 64 * i + (__ffsll((unsigned long long)x) - 1);
  }
  return res;
}
template <int NW>
SDX_DEV bool m_test(const M<NW>& a, int p) {
  return (m_word(a, p >> 6) >> (p & 63)) & 1ull;
}
template <int NW>
SDX_DEV bool m_any(const M<NW>& a) {
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) x |= a.w[i];
  return x != 0;
}

// positions where the packed-id string `tgt` (tlen chars) occurs: AND of shifted id bitmaps
template <int NW>
SDX_DEV M<NW> m_occ(const uint64_t* bm, uint64_t tgt, int tlen) {
  M<NW> acc = m_all<NW>();
  for (int i = 0; i < tlen; ++i) {
    const int id = (int)((tgt >> (4 * i)) & 15);
    M<NW> b;
#pragma unroll
    for (int k = 0; k < NW; ++k) b.w[k] = bm[id * NW + k];
    acc = m_and(acc, m_shr(b, i));  // i < 64: the word-aligned branch is never taken
  }
  return acc;
}

// ---------------------------------------------------------------------------------------------
// pattern_exists (pattern_utils.py:34-136) for one lane; fast path = one candidate per value
// ---------------------------------------------------------------------------------------------
// pair-presence bit of ids (a, b): set iff "ab" occurs in the message (TileLds::pairs)
struct PairRef {  // held in registers (reading the LDS row at each use measured 1.7 % slower)
  uint64_t P0, P1;
};
SDX_DEV bool pair_bit(const PairRef& P, int a, int b) {
  const int q = 10 * a + b;
  return ((q < 64 ? P.P0 >> q : P.P1 >> (q - 64)) & 1ull) != 0;
}

// one search list as the lane filter reads it (wave-uniform, scalar registers): from the full
// sdx_patspec or from the compact sdx_fspec of an sdx_mu_filt record
struct SpecV {
  int nu, slen;
  int klo[SDX_MAXUNIQ], khi[SDX_MAXUNIQ];
  uint32_t rk_off[SDX_MAXUNIQ];
  uint64_t upk;
};
SDX_DEV SpecV spec_full(const sdx_patspec* sp) {
  SpecV v;
  v.nu = cld(&sp->nuniq);
  v.slen = cld(&sp->len);
#pragma unroll
  for (int u = 0; u < SDX_MAXUNIQ; ++u) {
    v.klo[u] = cld(&sp->klo[u]);
    v.khi[u] = cld(&sp->khi[u]);
    v.rk_off[u] = cld(&sp->rk_off[u]);
  }
  v.upk = cld(&sp->uidx_pk);
  return v;
}
SDX_DEV SpecV spec_compact(const sdx_fspec* fs, uint64_t upk) {
  SpecV v;
  const uint32_t w = cld(&fs->rk2_len_nu), rk01 = cld(&fs->rk01);
  v.nu = (int)(w >> 24);
  v.slen = (int)((w >> 16) & 0xFF);
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const uint32_t lh = cld(&fs->lohi[u]);
    v.klo[u] = (int)(int16_t)(lh & 0xFFFF);
    v.khi[u] = (int)(int16_t)(lh >> 16);
  }
  v.klo[3] = 0;
  v.khi[3] = -1;
  v.rk_off[0] = rk01 & 0xFFFF;
  v.rk_off[1] = rk01 >> 16;
  v.rk_off[2] = w & 0xFFFF;
  v.rk_off[3] = 0;
  v.upk = upk;
  return v;
}

// rank key of candidate slot j for one search value: (gap rank << 4) | j -- the stable sort key of
// pattern_utils.py:61-63 (equal fp64 gaps share a rank; ties keep dict order j)
SDX_DEV uint32_t rank_key(const uint16_t* rt, int kqj, int klo, int j) {
  return ((uint32_t)rt[kqj - klo] << 4) | (uint32_t)j;
}
// the candidate of mask m (non-empty) that comes first in the sorted candidate list: one rank load
// per candidate, none when m has one bit
SDX_DEV int first_cand(uint32_t m, const int* kq, int klo, const uint16_t* rt) {
  if (!(m & (m - 1))) return __ffs(m) - 1;
  uint32_t best = 0xFFFFFFFFu;
#pragma unroll
  for (int j = 0; j < SDX_MAXPAT; ++j)
    if ((m >> j) & 1u) {
      const uint32_t k = rank_key(rt, kq[j], klo, j);
      best = k < best ? k : best;
    }
  return (int)(best & 15u);
}

template <int NW>
SDX_DEV PexRes pexists_lane(const SpecV& sp, const int* kq, uint64_t ids, int npat, const uint64_t* bm, int minpos,
                            const uint16_t* ranks, const PairRef& PR, bool need_pos) {
  PexRes res{false, -1, 0};
  const int nu = sp.nu, slen = sp.slen;
  // candidate slots per unique search value (pattern_utils.py:53-61) as an exact integer interval
  // test on k (bank.py _k_interval); kq[j] == SDX_K_NONE for j >= npat
  uint32_t okm[SDX_MAXUNIQ];
  int cnt[SDX_MAXUNIQ];
  long long total = 1;
#pragma unroll
  for (int u = 0; u < SDX_MAXUNIQ; ++u) {
    okm[u] = 0;
    cnt[u] = 1;
    if (u < nu) {
      const int klo = sp.klo[u], khi = sp.khi[u];
      uint32_t m = 0;
#pragma unroll
      for (int j = 0; j < SDX_MAXPAT; ++j) m |= (k_in(kq[j], klo, khi) ? 1u : 0u) << j;
      if (!m) return res;  // pattern_utils.py:78-80
      okm[u] = m;
      cnt[u] = __popc(m);
      total *= cnt[u];
      if (total > 10000) total = 10001;
    }
  }
  if (nu == 0 || total > 10000) return res;  // pattern_utils.py:93-101
  const uint64_t upk = sp.upk;
  // The first hit in itertools.product order (lexicographic in the sorted candidate lists) is
  // found without sorting for the two common shapes: (a) a 2-pulse search of two distinct values
  // (width-2 one/zero keys, 2-pulse starts) -- a* = the first-sorted a that has any valid partner,
  // b* = the first-sorted valid partner of a*; (b) a 1-pulse search -- the first-sorted a whose id
  // occurs.  Ranks are loaded only for the candidates that compete.
  if (nu == 2 && slen == 2 && upk == 0x10ull) {
    const bool cheap = minpos == 0 && !need_pos;  // pair presence decides exactly
    auto valid = [&](int a, int b, int* pos) -> bool {
      const int ida = (int)((ids >> (4 * a)) & 15), idb = (int)((ids >> (4 * b)) & 15);
      if (!pair_bit(PR, ida, idb)) return false;  // "ab" occurs nowhere
      if (cheap) {
        *pos = 0;
        return true;
      }
      *pos = m_first(m_occ<NW>(bm, (uint64_t)ida | ((uint64_t)idb << 4), 2), minpos);
      return *pos >= 0;
    };
    // the position of the last valid pair tested is kept: in the common case of one candidate
    // per value the pair is tested once (no re-test for b* or for the position)
    uint32_t va = 0;
    int b_last = -1, pos_last = -1;
    for (uint32_t ma = okm[0]; ma; ma &= ma - 1) {
      const int a = __ffs(ma) - 1;
      for (uint32_t mb = okm[1] & ~(1u << a); mb; mb &= mb - 1) {
        int p;
        if (valid(a, __ffs(mb) - 1, &p)) {
          va |= 1u << a;
          b_last = __ffs(mb) - 1;
          pos_last = p;
          break;
        }
      }
    }
    if (!va) return res;
    int a, b, pos_of_first;
    const uint32_t others_of = okm[1];
    if (!(va & (va - 1))) {
      a = __ffs(va) - 1;
      const uint32_t others = others_of & ~(1u << a);
      if (!(others & (others - 1))) {  // a single partner: the pair found above
        b = b_last;
        pos_of_first = pos_last;
      } else {
        b = -1;
      }
    } else {
      a = first_cand(va, kq, sp.klo[0], ranks + sp.rk_off[0]);
      b = -1;
    }
    if (b < 0) {
      uint32_t vb = 0;
      int nvb = 0;
      for (uint32_t mb = others_of & ~(1u << a); mb; mb &= mb - 1) {
        int p;
        if (valid(a, __ffs(mb) - 1, &p)) {
          vb |= 1u << (__ffs(mb) - 1);
          pos_last = p;
          ++nvb;
        }
      }
      b = first_cand(vb, kq, sp.klo[1], ranks + sp.rk_off[1]);
      if (nvb == 1) pos_of_first = pos_last;
      else if (need_pos) valid(a, b, &pos_of_first);
      else pos_of_first = 0;  // only found / tgt are read when the position is not needed
    }
    const int ida = (int)((ids >> (4 * a)) & 15), idb = (int)((ids >> (4 * b)) & 15);
    res.found = true;
    res.tgt = (uint64_t)ida | ((uint64_t)idb << 4);
    res.pos = pos_of_first;  // meaningful only with need_pos
    return res;
  }
  if (nu == 1 && slen == 1) {
    uint32_t va = 0;
    int pos_last = -1;
    for (uint32_t ma = okm[0]; ma; ma &= ma - 1) {
      const int a = __ffs(ma) - 1, ida = (int)((ids >> (4 * a)) & 15);
      const int p = m_first(m_occ<NW>(bm, (uint64_t)ida, 1), minpos);
      if (p >= 0) {
        va |= 1u << a;
        pos_last = p;
      }
    }
    if (!va) return res;
    const int a = first_cand(va, kq, sp.klo[0], ranks + sp.rk_off[0]);
    res.found = true;
    res.tgt = (ids >> (4 * a)) & 15;
    res.pos = (va & (va - 1)) ? m_first(m_occ<NW>(bm, res.tgt, 1), minpos) : pos_last;
    return res;
  }
  // general shape: the sorted candidate lists (packed nibbles), then the product loop
  uint64_t cand[SDX_MAXUNIQ];
#pragma unroll
  for (int u = 0; u < SDX_MAXUNIQ; ++u) {
    cand[u] = 0;
    if (u < nu) {
      if (cnt[u] == 1) {
        cand[u] = (uint64_t)(__ffs(okm[u]) - 1);
      } else {  // stable sort by the fp64 gap of k/10 (bank gap-rank table), ties in dict order
        const uint16_t* rt = ranks + sp.rk_off[u];
        const int klo = sp.klo[u];
        uint32_t key[SDX_MAXPAT];
#pragma unroll
        for (int j = 0; j < SDX_MAXPAT; ++j)
          key[j] = ((okm[u] >> j) & 1u) ? rank_key(rt, kq[j], klo, j) : 0xFFFFFFFFu;
        sort10(key);
        uint64_t packed = 0;
#pragma unroll
        for (int i = 0; i < SDX_MAXPAT; ++i)
          packed |= (i < cnt[u]) ? (uint64_t)(key[i] & 15u) << (4 * i) : 0ull;
        cand[u] = packed;
      }
    }
  }
  int digit[SDX_MAXUNIQ];
#pragma unroll
  for (int u = 0; u < SDX_MAXUNIQ; ++u) digit[u] = 0;
  for (long long it = 0; it < total; ++it) {
    uint32_t used = 0, uid = 0;
    bool dup = false;
#pragma unroll
    for (int u = 0; u < SDX_MAXUNIQ; ++u) {
      if (u < nu) {
        const int slot = (int)((cand[u] >> (4 * digit[u])) & 15);
        if (used & (1u << slot)) dup = true;
        used |= 1u << slot;
        uid |= (uint32_t)((ids >> (4 * slot)) & 15) << (4 * u);
      }
    }
    if (!dup) {
      uint64_t tgt = 0;
      for (int i = 0; i < slen; ++i) tgt |= (uint64_t)((uid >> (4 * (int)((upk >> (4 * i)) & 15))) & 15) << (4 * i);
      // every adjacent id pair of the target must occur in the message: exact for a 2-id target
      // searched from position 0, a necessary condition otherwise
      bool ok = true;
      for (int i = 0; i + 1 < slen; ++i)
        ok = ok && pair_bit(PR, (int)((tgt >> (4 * i)) & 15), (int)((tgt >> (4 * i + 4)) & 15));
      int p = -1;
      if (ok) p = (slen == 2 && minpos == 0 && !need_pos) ? 0 : m_first(m_occ<NW>(bm, tgt, slen), minpos);
      if (p >= 0) {
        res.found = true;
        res.pos = p;
        res.tgt = tgt;
        return res;
      }
    }
#pragma unroll
    for (int u = SDX_MAXUNIQ - 1; u >= 0; --u) {
      if (u < nu) {
        if (digit[u] + 1 < cnt[u]) {
          digit[u]++;
          break;
        }
        digit[u] = 0;
      }
    }
  }
  return res;
}

// bits [0, k)
template <int NW>
SDX_DEV M<NW> m_range_lo(int k) {
  M<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int hi = k - 64 * i;
    r.w[i] = hi >= 64 ? ~0ull : (hi <= 0 ? 0ull : ((1ull << hi) - 1));
  }
  return r;
}
// set bit b of a packed bitstring (branch-free per word)
template <int NW>
SDX_DEV void m_set(M<NW>& a, int b) {
  const uint64_t bitv = 1ull << (b & 63);
  const int wi = b >> 6;
#pragma unroll
  for (int i = 0; i < NW; ++i) a.w[i] |= bitv & (0ull - (uint64_t)(wi == i));
}
// len (<= 4) bits starting at b, first bit = most significant (int(''.join(bits[b:b+len]), 2))
template <int NW>
SDX_DEV int m_nibble(const M<NW>& a, int b, int len) {
  const uint64_t lo = m_word(a, b >> 6), hi = m_word(a, (b >> 6) + 1);
  const int sh = b & 63;
  const uint32_t x = (uint32_t)((sh ? ((lo >> sh) | (hi << (64 - sh))) : lo) & 15u);
  const uint32_t r4 = ((x & 1u) << 3) | ((x & 2u) << 1) | ((x & 4u) >> 1) | ((x & 8u) >> 3);
  return (int)(r4 >> (4 - len));
}

// positions congruent to r modulo L (L in {1,2,4,8,16}: 64 % L == 0)
SDX_DEV uint64_t residue_word(int L, int r) {
  uint64_t m = 0;
  switch (L) {
    case 1: m = ~0ull; break;
    case 2: m = 0x5555555555555555ull; break;
    case 4: m = 0x1111111111111111ull; break;
    case 8: m = 0x0101010101010101ull; break;
    default: m = 0x0001000100010001ull; break;
  }
  return m << r;
}

// "a run of >= m units (stride L) starts here": AND_{j<m} (U >> jL), by doubling
template <int NW>
SDX_DEV M<NW> m_runs(const M<NW>& U, int m, int L) {
  M<NW> res = m_all<NW>();
  int res_len = 0, cur_len = 1;
  M<NW> cur = U;
  while (m) {
    if (m & 1) {
      res = m_and(res, m_shr(cur, res_len * L));
      res_len += cur_len;
    }
    m >>= 1;
    if (m) {
      cur = m_and(cur, m_shr(cur, cur_len * L));
      cur_len *= 2;
    }
  }
  return res;
}

// compact every L-th bit (L in {1,2,4}) of a 64-bit word into its low 64/L bits
SDX_DEV uint64_t compact_stride(uint64_t x, int L) {
  if (L == 2) {
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
  } else if (L == 4) {
    x &= 0x1111111111111111ull;
    x = (x | (x >> 3)) & 0x0303030303030303ull;
    x = (x | (x >> 6)) & 0x000F000F000F000Full;
    x = (x | (x >> 12)) & 0x000000FF000000FFull;
    x = (x | (x >> 24)) & 0x000000000000FFFFull;
  }
  return x;
}

// packed bit i = A bit (q + i*L), i < k (L in {1,2,4})
template <int NW>
SDX_DEV M<NW> m_stride_extract(const M<NW>& A, int q, int L, int k) {
  const M<NW> B = m_shr(A, q);
  M<NW> P = m_zero<NW>();
  if (L == 1) {
    P = B;
  } else {
    const int per = 64 / L;  // packed bits contributed by one source word
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint64_t c = compact_stride(B.w[w], L);
      const int bitpos = w * per;
#pragma unroll
      for (int o = 0; o < NW; ++o) {
        const int lo = bitpos - 64 * o;
        if (lo >= 0 && lo < 64) P.w[o] |= c << lo;
        else if (lo < 0 && lo > -64) P.w[o] |= c >> (-lo);
      }
    }
  }
  return m_and(P, m_range_lo<NW>(k));
}

}  // namespace sdx
