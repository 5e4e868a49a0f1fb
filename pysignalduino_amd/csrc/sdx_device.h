// sdx_device.h -- device-side building blocks of the MU/MS/MC demodulator (gfx950).
//
// Everything here is plain integer / fp64 work: no MFMA (the path is
// compares, substring tests and bit packing, not a contraction).  Bit-exactness
// with the reference Python (RFD-FHEM/PySignalduino sd_protocols/*) is the
// first requirement; the file is compiled with -ffp-contract=off so that
// e.g. abs(pc - clk) > clk*0.3 is evaluated with exactly Python's roundings.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sdx.h"
#include "../../include/sdx_bank.h"

#define SDX_DEV __device__ __forceinline__

// MS tiles of short messages on the NW = SDX_MS_NARROW_W instantiation of k_pulses (sdx_kernels.hip
// sdx_demod_pulses; the MS grouping key's top bit separates them, sdx_group.hip k_sig)
#ifndef SDX_MS_NARROW
#define SDX_MS_NARROW 1  /* MS length classes <= 128 / <= 256 pulses */
#endif

namespace sdx {

constexpr int WAVE = 64;

// ------------------------------------------------------------------------------------------------
// Python round(x, 1): correctly rounded to one decimal, ties to even on the EXACT binary value,
// then the nearest double to that decimal (message_unsynced.py:64, message_synced.py:72).
// k = round_half_even(10*x) is decided with fma() residuals, which carry the exact sign of
// 10x - c; k/10.0 is the correctly rounded quotient = the double Python's strtod returns.
// |x| >= 2^49: x is a multiple of 1/8 and |k/10 - x| <= 0.05 < ulp(x)/2, so round(x,1) == x.
// NaN / inf are returned unchanged, like Python.
// ------------------------------------------------------------------------------------------------
SDX_DEV double py_round1(double q) {
  if (!(fabs(q) < 562949953421312.0)) return q;  // 2^49, also NaN / inf
  double f = floor(q * 10.0);
  if (fma(10.0, q, -f) < 0.0) f -= 1.0;
  else if (fma(10.0, q, -(f + 1.0)) >= 0.0) f += 1.0;
  const double r = fma(10.0, q, -(f + 0.5));
  double k;
  if (r > 0.0) k = f + 1.0;
  else if (r < 0.0) k = f;
  else k = (((long long)f & 1) == 0) ? f : f + 1.0;  // |f| < 2^53: exact parity
  double res = k / 10.0;
  if (res == 0.0) res = copysign(0.0, q);
  return res;
}

// the integer k of py_round1(q) == k / 10.0, or SDX_K_NONE when |q| >= 2^26 / NaN / inf: such a
// value lies outside every bank interval [klo, khi] (bank.py bounds them by 2^28), exactly as its
// fp64 gap exceeds every tolerance
constexpr int SDX_K_NONE = INT32_MIN;
SDX_DEV int py_round1_k(double q) {
  if (!(fabs(q) < 67108864.0)) return SDX_K_NONE;
  double f = floor(q * 10.0);
  if (fma(10.0, q, -f) < 0.0) f -= 1.0;
  else if (fma(10.0, q, -(f + 1.0)) >= 0.0) f += 1.0;
  const double r = fma(10.0, q, -(f + 0.5));
  double k;
  if (r > 0.0) k = f + 1.0;
  else if (r < 0.0) k = f;
  else k = (((long long)f & 1) == 0) ? f : f + 1.0;  // |f| < 2^53: exact parity
  return (int)k;
}
// 10-key sorting network (29 comparators, depth 8; Knuth TAOCP 5.3.4), ascending
SDX_DEV void sort10(uint32_t* a) {
#define SDX_CE(i, j)                      \
  {                                       \
    const uint32_t x = a[i], y = a[j];    \
    a[i] = x < y ? x : y;                 \
    a[j] = x < y ? y : x;                 \
  }
  SDX_CE(4, 9) SDX_CE(3, 8) SDX_CE(2, 7) SDX_CE(1, 6) SDX_CE(0, 5) SDX_CE(1, 4) SDX_CE(6, 9) SDX_CE(0, 3)
  SDX_CE(5, 8) SDX_CE(0, 2) SDX_CE(3, 6) SDX_CE(7, 9) SDX_CE(0, 1) SDX_CE(2, 4) SDX_CE(5, 7) SDX_CE(8, 9)
  SDX_CE(1, 2) SDX_CE(4, 6) SDX_CE(7, 8) SDX_CE(3, 5) SDX_CE(2, 5) SDX_CE(6, 8) SDX_CE(1, 3) SDX_CE(4, 7)
  SDX_CE(2, 3) SDX_CE(6, 7) SDX_CE(3, 4) SDX_CE(5, 6) SDX_CE(4, 5)
#undef SDX_CE
}

// klo <= k <= khi (SDX_K_NONE never passes: the unsigned difference exceeds any interval width)
SDX_DEV bool k_in(int k, int klo, int khi) { return (uint32_t)k - (uint32_t)klo <= (uint32_t)khi - (uint32_t)klo; }

// ------------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------------
SDX_DEV int lane_id() { return __lane_id(); }
SDX_DEV uint64_t ballot(bool p) { return __ballot(p); }
SDX_DEV int bcast_i(int v, int src) { return __shfl(v, src); }
SDX_DEV uint64_t bcast_u64(uint64_t v, int src) {
  uint32_t lo = __shfl((uint32_t)v, src), hi = __shfl((uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
SDX_DEV int ffs64(uint64_t x) { return __ffsll((unsigned long long)x) - 1; }  // -1 if zero
SDX_DEV int popc64(uint64_t x) { return __popcll(x); }

// bits p..p+63 of a position bitmap (bit i of word w = position 64w+i), reading words w and w+1
SDX_DEV uint64_t bm_window(const uint64_t* bm, int w, int sh, int nw) {
  uint64_t lo = bm[w];
  if (sh == 0) return lo;
  uint64_t hi = (w + 1 < nw) ? bm[w + 1] : 0ull;
  return (lo >> sh) | (hi << (64 - sh));
}

// ------------------------------------------------------------------------------------------------
// pattern_exists (pattern_utils.py:34-136), one lane = one message.
//   kq[] / ids:   the message's normalised pattern values (as k of k/10) and their id digits
//                 in dict order
//   bm:           the message's per-id position bitmaps, bm[id*ws + w]
// Returns the first id assignment (itertools.product order over gap-sorted candidate lists,
// no id reused) whose concatenation occurs at a position >= minpos; tgt = its id digits packed
// 4 bits per character, pos = first occurrence (str.find).  found=false <=> the reference's -1.
// ------------------------------------------------------------------------------------------------
struct PexRes {
  bool found;
  int pos;
  uint64_t tgt;
};

SDX_DEV bool substr_first(const uint64_t* bm, int ws, int nw, uint64_t tgt, int tlen, int minpos, int* pos) {
  for (int w = minpos >> 6; w < nw; ++w) {
    uint64_t acc = ~0ull;
    for (int i = 0; i < tlen && acc; ++i) {
      const int id = (int)((tgt >> (4 * i)) & 15);
      // position p = 64w+b matches char i iff bit (p+i) of bm[id] is set
      const int sh = i & 63, wo = w + (i >> 6);
      uint64_t v = 0;
      if (wo < nw) v = bm_window(bm + id * ws, wo, sh, nw);
      acc &= v;
    }
    if (w == (minpos >> 6) && (minpos & 63)) acc &= ~0ull << (minpos & 63);
    if (acc) {
      *pos = w * 64 + ffs64(acc);
      return true;
    }
  }
  return false;
}

__device__ __noinline__ PexRes pattern_exists(const sdx_patspec* sp, const int* kq, uint64_t ids, int npat,
                                              const uint64_t* bm, int ws, int nw, int minpos) {
  PexRes res{false, -1, 0};
  const int nu = sp->nuniq, slen = sp->len;
  uint64_t cand[SDX_MAXUNIQ];
  int cnt[SDX_MAXUNIQ];
  long long total = 1;
#pragma unroll
  for (int u = 0; u < SDX_MAXUNIQ; ++u) {
    cand[u] = 0;
    cnt[u] = 1;
    if (u < nu) {
      const double v = sp->uval[u];
      const int klo = sp->klo[u], khi = sp->khi[u];
      double gap[SDX_MAXPAT];
      bool ok[SDX_MAXPAT];
#pragma unroll
      for (int j = 0; j < SDX_MAXPAT; ++j) {
        ok[j] = (j < npat) && k_in(kq[j], klo, khi);  // == (gap <= 0.001 or gap <= tol)
        gap[j] = fabs((double)kq[j] / 10.0 - v);        // the fp64 gap of norm == k/10 (ranking only)
      }
      int c = 0;
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < SDX_MAXPAT; ++j) {
        if (ok[j]) {
          int rank = 0;  // stable sort by gap (list.sort is stable; dict order breaks ties)
#pragma unroll
          for (int k = 0; k < SDX_MAXPAT; ++k)
            rank += (ok[k] && (gap[k] < gap[j] || (gap[k] == gap[j] && k < j))) ? 1 : 0;
          packed |= (uint64_t)j << (4 * rank);
          ++c;
        }
      }
      cand[u] = packed;
      cnt[u] = c;
      total *= c;
      if (total > 10000) total = 10001;  // saturate: > 10000 combinations -> -1 (:97-101)
    }
  }
  if (nu == 0) return res;
  for (int u = 0; u < nu; ++u)
    if (cnt[u] == 0) return res;
  if (total > 10000) return res;
  // itertools.product order: the LAST unique value varies fastest
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
      for (int i = 0; i < slen; ++i) tgt |= (uint64_t)((uid >> (4 * sp->uidx[i])) & 15) << (4 * i);
      int pos;
      if (substr_first(bm, ws, nw, tgt, slen, minpos, &pos)) {
        res.found = true;
        res.pos = pos;
        res.tgt = tgt;
        return res;
      }
    }
    // advance the mixed-radix counter
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

// test one string (packed id digits) at an absolute position against the bitmaps
SDX_DEV bool match_at(const uint64_t* bm, int ws, int n, uint64_t tgt, int tlen, int x) {
  if (x < 0 || x + tlen > n) return false;
  for (int i = 0; i < tlen; ++i) {
    const int id = (int)((tgt >> (4 * i)) & 15), p = x + i;
    if (!((bm[id * ws + (p >> 6)] >> (p & 63)) & 1ull)) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------------------------
// postDemodulation functions (postdemodulation.py), single lane, bits as 0/1 bytes.
// return 1 = (1, bits), 0 = (0, None), -1 = the reference raises ValueError (int('', 2)).
// ------------------------------------------------------------------------------------------------
SDX_DEV int bval(const uint8_t* b, int a, int e) {  // int(''.join(bits[a:e]), 2), e - a <= 31
  int v = 0;
  for (int i = a; i < e; ++i) v = (v << 1) | b[i];
  return v;
}
SDX_DEV int first_one(const uint8_t* b, int n) {
  for (int i = 0; i < n; ++i)
    if (b[i] == 1) return i;
  return -1;
}

// postdemodulation.py:27-88
SDX_DEV int pd_em(const uint8_t* b, int n, uint8_t* o, int* no) {
  int p = -1;
  for (int i = 0; i + 10 <= n; ++i) {
    bool ok = b[i + 9] == 1;
    for (int j = 0; ok && j < 9; ++j) ok = b[i + j] == 0;
    if (ok) { p = i; break; }
  }
  if (p < 0) return 0;
  const uint8_t* s = b + p + 10;
  const int m = n - p - 10;
  if (m != 89) return 0;
  int crc = 0, k = 0;
  for (int c = 0; c + 8 < m; c += 9) {
    if (c < m - 10) {
      for (int j = 7; j >= 0; --j) o[k++] = s[c + j];
      crc ^= bval(s, c, c + 8);
    }
  }
  if (crc != bval(s, m - 8, m)) return 0;
  *no = k;
  return 1;
}

// postdemodulation.py:90-137
SDX_DEV int pd_revolt(const uint8_t* b, int n, uint8_t* o, int* no) {
  if (n < 96) return 0;
  int sum = 0;
  for (int i = 0; i < 88; i += 8) sum += bval(b, i, i + 8);
  if ((sum & 0xFF) != bval(b, 88, 96)) return 0;
  for (int i = 0; i < 88; ++i) o[i] = b[i];
  *no = 88;
  return 1;
}

// parity of every 9-bit group even; copy the 8 data bits of group g to o
SDX_DEV bool groups9_even(const uint8_t* m, int k) {
  for (int g = 0; g < k; g += 9) {
    int par = 0;
    for (int i = g; i < g + 9 && i < k; ++i) par += m[i];
    if (par & 1) return false;
  }
  return true;
}

// postdemodulation.py:139-243
SDX_DEV int pd_fs20(const uint8_t* b, int n, uint8_t* o, int* no) {
  const int st = first_one(b, n);
  if (st < 0) return 0;
  const uint8_t* m = b + st + 1;
  int k = n - st - 1;
  if (k == 46 || k == 55) --k;
  if (k != 45 && k != 54) return 0;
  int sum = 6;
  for (int g = 0; g < k - 9; g += 9) sum += bval(m, g, g + 8);
  const int chk = bval(m, k - 9, k - 1);
  if (((sum + 6) & 0xFF) == chk) return 0;
  if ((sum & 0xFF) != chk) return 0;
  if (!groups9_even(m, k)) return 0;
  const int nbytes = k / 9;  // 5 or 6 data bytes incl. checksum
  int q = 0;
  for (int g = 0; g < nbytes; ++g) {
    if (k == 45 && g == 3) for (int j = 0; j < 8; ++j) o[q++] = 0;  // insert 8 zeros at 24
    if (g == nbytes - 1) break;                                    // drop the checksum byte
    for (int j = 0; j < 8; ++j) o[q++] = m[9 * g + j];
  }
  *no = q;
  return 1;
}

// postdemodulation.py:245-337
SDX_DEV int pd_fht80(const uint8_t* b, int n, uint8_t* o, int* no) {
  const int st = first_one(b, n);
  if (st < 0) return 0;
  const uint8_t* m = b + st + 1;
  int k = n - st - 1;
  if (k == 55) --k;
  if (k != 54) return 0;
  int sum = 12;
  for (int g = 0; g < 45; g += 9) sum += bval(m, g, g + 8);
  const int chk = bval(m, 45, 53);
  if (((sum - 6) & 0xFF) == chk) return 0;
  if ((sum & 0xFF) != chk) return 0;
  if (!groups9_even(m, 54)) return 0;
  int q = 0;
  for (int g = 0; g < 6; ++g)
    for (int j = 0; j < 8; ++j) o[q++] = m[9 * g + j];
  *no = q;
  return 1;
}

// postdemodulation.py:339-423
SDX_DEV int pd_fht80tf(const uint8_t* b, int n, uint8_t* o, int* no) {
  if (n < 46) return 0;
  const int st = first_one(b, n);
  if (st < 0) return 0;
  const uint8_t* m = b + st + 1;
  const int k = n - st - 1;
  if (k != 45) return 0;
  int sum = 12;
  for (int g = 0; g < 36; g += 9) sum += bval(m, g, g + 8);
  if ((sum & 0xFF) != bval(m, 36, 44)) return 0;
  if (!groups9_even(m, 45)) return 0;
  // after removing the 5 parity bits: 40 bits d0..d4; bit 26 must be 0; drop d4
  if (m[9 * 3 + 2] != 0) return 0;
  int q = 0;
  for (int g = 0; g < 4; ++g)
    for (int j = 0; j < 8; ++j) o[q++] = m[9 * g + j];
  *no = q;
  return 1;
}

// postdemodulation.py:425-578
SDX_DEV int rev_nib(const uint8_t* b, int a, int e) {  // int(''.join(reversed(bits[a:e])), 2)
  int v = 0;
  for (int i = e - 1; i >= a; --i) v = (v << 1) | b[i];
  return v;
}
SDX_DEV int pd_ws2000(const uint8_t* b, int n, uint8_t* o, int* no) {
  const int st = first_one(b, n);
  if (st < 0) return 0;
  const int dlen = n - st;
  int dlen1 = dlen - dlen % 5;
  const int te = (st + 5 < n) ? st + 5 : n;
  if (te <= st + 1) return -1;  // int('', 2) -> ValueError
  const int typ = rev_nib(b, st + 1, te);
  if (typ > 7) return 0;
  if (typ == 1 && (dlen == 45 || dlen == 46)) dlen1 += 5;
  const int tab[8] = {35, 50, 35, 50, 70, 40, 40, 85};
  if (tab[typ] != dlen1) return 0;
  if (st > 10) return 0;
  int idx = 0, didx = 0, check = 0, acc = 5;
  while (idx < dlen - 1) {
    if (b[idx + st] != 1) return 0;
    didx = idx + st + 1;
    if (n - didx < 4) return 0;
    const int nib = rev_nib(b, didx, didx + 4);
    if (dlen == 45 || dlen == 46) {
      if (idx <= dlen - 5) check ^= nib;
    } else if (idx <= dlen - 10) {
      check ^= nib;
      acc += nib;
    }
    idx += 5;
  }
  if (check != 0) return 0;
  if (dlen < 45 || dlen > 46) {
    const int e = (didx + 4 < n) ? didx + 4 : n;
    if (e <= didx) return -1;
    if (rev_nib(b, didx, e) != (acc & 0x0F)) return 0;
  }
  const int d = st + 1;
  int q = 0;
  auto rv = [&](int a, int e) {
    for (int i = d + e - 1; i >= d + a; --i)
      if (i < n) o[q++] = b[i];
  };
  rv(5, 9); rv(0, 4); rv(15, 19); rv(10, 14);
  if (typ == 0 || typ == 2) {
    rv(20, 24);
  } else if (typ == 1 || typ == 3 || typ == 4 || typ == 7) {
    rv(25, 29); rv(20, 24); rv(35, 39); rv(30, 34);
    if (typ == 4) { rv(55, 59); rv(50, 54); rv(45, 49); rv(40, 44); }
  }
  *no = q;
  return 1;
}

// postdemodulation.py:580-640
SDX_DEV int pd_ws7035(const uint8_t* b, int n, uint8_t* o, int* no) {
  if (n < 8) return 0;
  const uint8_t ident[8] = {1, 0, 1, 0, 0, 0, 0, 0};
  for (int i = 0; i < 8; ++i)
    if (b[i] != ident[i]) return 0;
  if (n != 44) return 0;
  int par = 0;
  for (int i = 15; i < 28; ++i) par += b[i];
  if (par & 1) return 0;
  int s = 0;
  for (int i = 0; i < 40; i += 4) s += bval(b, i, i + 4);
  if ((s % 16) != bval(b, 40, 44)) return 0;
  int q = 0;
  for (int i = 0; i < 44; ++i)
    if (i < 27 || i >= 31) o[q++] = b[i];
  *no = q;
  return 1;
}

// postdemodulation.py:642-706
SDX_DEV int pd_ws7053(const uint8_t* b, int n, uint8_t* o, int* no) {
  int p = -1;
  const uint8_t ident[8] = {1, 0, 1, 0, 0, 0, 0, 0};
  for (int i = 0; i + 8 <= n && p < 0; ++i) {
    bool ok = true;
    for (int j = 0; ok && j < 8; ++j) ok = b[i + j] == ident[j];
    if (ok) p = i;
  }
  if (p < 0) return 0;
  const uint8_t* s = b + (p > 0 ? p : 0);
  const int len = (p > 0) ? n - p + 1 : n;  // s[p:] + "0"
  auto at = [&](int i) -> int { return (p > 0 && i == len - 1) ? 0 : s[i]; };
  if (len < 32) return 0;
  int par = 0;
  for (int i = 15; i < 28; ++i) par += at(i);
  if (par & 1) return 0;
  int q = 0;
  for (int i = 0; i < 28; ++i) o[q++] = at(i);
  for (int i = 16; i < 24; ++i) o[q++] = at(i);
  for (int i = 28; i < 32; ++i) o[q++] = at(i);
  *no = q;
  return 1;
}

// postdemodulation.py:708-730  (format(len, '08b') grows past 8 bits for len >= 256)
SDX_DEV int pd_lenprefix(const uint8_t* b, int n, uint8_t* o, int* no) {
  int nb = 8;
  while ((n >> nb) != 0) ++nb;
  int q = 0;
  for (int i = nb - 1; i >= 0; --i) o[q++] = (n >> i) & 1;
  for (int i = 0; i < n; ++i) o[q++] = b[i];
  *no = q;
  return 1;
}

SDX_DEV int run_postdemo(int which, const uint8_t* b, int n, uint8_t* o, int* no) {
  switch (which) {
    case SDX_PD_EM: return pd_em(b, n, o, no);
    case SDX_PD_REVOLT: return pd_revolt(b, n, o, no);
    case SDX_PD_FS20: return pd_fs20(b, n, o, no);
    case SDX_PD_FHT80: return pd_fht80(b, n, o, no);
    case SDX_PD_FHT80TF: return pd_fht80tf(b, n, o, no);
    case SDX_PD_WS2000: return pd_ws2000(b, n, o, no);
    case SDX_PD_WS7035: return pd_ws7035(b, n, o, no);
    case SDX_PD_WS7053: return pd_ws7053(b, n, o, no);
    case SDX_PD_LENPREFIX: return pd_lenprefix(b, n, o, no);
  }
  return 0;
}

// ------------------------------------------------------------------------------------------------
// bank accessors.  Every bank pointer is made provably wave-uniform (readfirstlane), so the
// compiler reads protocol records with scalar loads into SGPRs instead of per-lane vector loads.
// ------------------------------------------------------------------------------------------------
// load through the constant address space: with a uniform address this is an s_load into SGPRs
template <class T>
SDX_DEV T cld(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}

template <class T>
SDX_DEV const T* uniform_ptr(const T* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const T*)(((uint64_t)hi << 32) | lo);
}
struct BankView {
  const uint8_t* base;
  const sdx_bank_hdr* hdr;
  const sdx_mu_proto* mu;
  const sdx_ms_proto* ms;
  const sdx_mc_proto* mc;
  const sdx_dfa* dfa;
  const uint8_t* cls;
  const uint16_t* trans;
  const uint8_t* t256;
  const uint8_t* dflags;
  const uint8_t* str;
  const uint16_t* order;  // processing order: MU indices, then MS indices
  const uint16_t* rank;   // candidate gap-rank tables
  const sdx_mu_desc* mudesc;
  const uint8_t* mmtab;
  const sdx_mu_filt* mufilt;  // compact MU lane-filter records (128 B each)
  const sdx_ms_filt* msfilt;  // compact MS lane-filter records
};

SDX_DEV BankView bank_view(const void* blob) {
  BankView v;
  v.base = uniform_ptr((const uint8_t*)blob);
  v.hdr = (const sdx_bank_hdr*)blob;
  v.mu = (const sdx_mu_proto*)(v.base + v.hdr->off_mu);
  v.ms = (const sdx_ms_proto*)(v.base + v.hdr->off_ms);
  v.mc = (const sdx_mc_proto*)(v.base + v.hdr->off_mc);
  v.dfa = (const sdx_dfa*)(v.base + v.hdr->off_dfa);
  v.cls = v.base + v.hdr->off_cls;
  v.trans = (const uint16_t*)(v.base + v.hdr->off_trans);
  v.t256 = v.base + v.hdr->off_t256;
  v.dflags = v.base + v.hdr->off_flags;
  v.str = v.base + v.hdr->off_str;
  v.order = (const uint16_t*)(v.base + v.hdr->off_order);
  v.rank = (const uint16_t*)(v.base + v.hdr->off_rank);
  v.mudesc = (const sdx_mu_desc*)(v.base + v.hdr->off_mudesc);
  v.mmtab = v.base + v.hdr->off_mmtab;
  v.mufilt = (const sdx_mu_filt*)(v.base + v.hdr->off_mufilt);
  v.msfilt = (const sdx_ms_filt*)(v.base + v.hdr->off_msfilt);
  v.hdr = uniform_ptr(v.hdr);
  v.mu = uniform_ptr(v.mu);
  v.ms = uniform_ptr(v.ms);
  v.mc = uniform_ptr(v.mc);
  v.dfa = uniform_ptr(v.dfa);
  v.cls = uniform_ptr(v.cls);
  v.trans = uniform_ptr(v.trans);
  v.t256 = uniform_ptr(v.t256);
  v.dflags = uniform_ptr(v.dflags);
  v.str = uniform_ptr(v.str);
  v.order = uniform_ptr(v.order);
  v.rank = uniform_ptr(v.rank);
  v.mudesc = uniform_ptr(v.mudesc);
  v.mmtab = uniform_ptr(v.mmtab);
  v.mufilt = uniform_ptr(v.mufilt);
  v.msfilt = uniform_ptr(v.msfilt);
  return v;
}

// re.search(modulematch, payload): continue the DFA from the preamble state over the rest
SDX_DEV bool dfa_accepts(const BankView& bv, int d, int state, const uint8_t* s, int n) {
  const sdx_dfa D = bv.dfa[d];
  const uint8_t* t256 = bv.t256 + D.t256_off;
  const uint8_t* fl = bv.dflags + D.flags_off;
  for (int i = 0; i < n; ++i) {
    const uint8_t f = fl[state];
    if (f & 1) return true;
    if (f & 4) return false;
    state = t256[state * 256 + s[i]];
  }
  const uint8_t f = fl[state];
  return (f & 3) != 0;
}

}  // namespace sdx
