// sdx_mc.h -- the Manchester (MC) protocol methods on the device, shared by the "fixed" MC chain
// (k_mc, sdx_kernels.hip) and the unit-level entry (k_units, sdx_units.hip).
//
// A frame's bit string lives in LDS as MSB-first 64-bit words, lane-strided (word w of lane t at
// base[w * 256], 256 threads per workgroup).  mc_method restates the reference's methods
// (sd_protocols/manchester.py:207-795, helpers.py:90-122) on that representation:
//   n  = len(bit_data)            -- every find / slice / hex conversion,
//   mb = the mcbitnum argument    -- every length gate (the chain passes len(bit_data), :120),
// and reports the reference's return value: rc 1 with a payload description, rc 0 for (-1, msg)
// with `why` naming msg (McWhy), or a raised exception class.
#pragma once
#include "sdx_device.h"

namespace sdx {

constexpr int MC_MAXW = 8;   // <= 512 bits = 128 hex characters per frame (device contract)
constexpr int MC_SHORTW = 4; // k_mc<4>: frames of <= 64 hex characters (the long variant takes the rest)

// the (-1, msg) texts of the methods; the host renders them (pysignalduino_amd/units.py MC_WHY)
enum McWhy {
  MCW_NONE = 0,
  MCW_SHORT = 1,        // 'message is too short'
  MCW_LONG = 2,         // 'message is too long'
  MCW_BEGIN = 3,        // 'wrong bits at begin' (Funkbus)
  MCW_PARITY = 4,       // 'parity error' (Funkbus)
  MCW_CHECKSUM = 5,     // 'checksum error' (Funkbus)
  MCW_SAIN_START = 6,   // f"{name}: lib/mcBit2Sainlogic, start 010100 not found"
  MCW_TFA_SYNC = 7,     // 'sync not found'
  MCW_TFA_LOOP = 8,     // f'loop error, please report this data {bit_data}'
  MCW_TFA_NODUP = 9,    // f' no duplicate found{retmsg}', aux = retmsg: 0 '', 1/2/3 ', ' + length_in_range text
  MCW_GROTHE = 10,      // f"message must be 32 bits, got {mcbitnum}"
  MCW_SOMFY = 11,       // f"message must be 56 bits, got {len(bit_data)}", aux = that length
  MCW_TO_LONG = 12      // 'message is to long' (helpers.mcraw)
};

// a frame's bit string, word w at base[w * 256] (words beyond nw read as 0).  dm: the Funkbus
// mc2dmc(lh/hl) view of the same words, bit k = (b[k] == b[k+1]) -- derived on the fly
struct LaneBits {
  const uint64_t* base;
  int nw;
  bool dm;
  SDX_DEV uint64_t raw(int w) const { return w < nw ? base[w * 256] : 0ull; }
  SDX_DEV uint64_t word(int w) const {
    const uint64_t x = raw(w);
    return dm ? (w < nw ? ~(x ^ ((x << 1) | (raw(w + 1) >> 63))) : 0ull) : x;
  }
  SDX_DEV int get(int i) const { return (int)((word(i >> 6) >> (63 - (i & 63))) & 1ull); }
  // P <= 32 bits starting at i (MSB-first), zero beyond the array
  SDX_DEV uint32_t win(int i, int P) const {
    const int w = i >> 6, o = i & 63;
    uint64_t hi = word(w) << o;
    if (o) hi |= word(w + 1) >> (64 - o);
    return (uint32_t)(hi >> (64 - P));
  }
  // str.find: first i >= from with bits [i, i+P) == pat and i + P <= n (P <= 32): 64 start
  // positions per step, matched bit-parallel on two words (two LDS reads per 64 positions)
  SDX_DEV int find(uint32_t pat, int P, int from, int n) const {
    if (from < 0) from = 0;
    for (int w = from >> 6; 64 * w + P <= n; ++w) {
      const uint64_t a = word(w), b = word(w + 1);
      uint64_t m = ~0ull;  // bit 63 - j: start 64w + j still matches
      for (int t = 0; t < P; ++t) {
        const uint64_t xt = t ? ((a << t) | (b >> (64 - t))) : a;  // bit 63 - j = string bit 64w + j + t
        m &= ((pat >> (P - 1 - t)) & 1u) ? xt : ~xt;
      }
      const int lo = from - 64 * w;  // j >= lo
      if (lo > 0) m &= ~0ull >> lo;
      const int hi = n - P - 64 * w;  // j <= hi
      if (hi < 63) m &= ~0ull << (63 - hi);
      if (m) return 64 * w + __clzll((long long)m);
    }
    return -1;
  }
};

// bin_str_2_hex_str of bits [a, e) of LaneBits -> dst; returns the length.  Digit d is
// int(bits[e - 4 (nd - d) : e - 4 (nd - 1 - d)], 2), the first one clipped at a; 8 digits per step:
// one 32-bit window (two LDS reads), nibble-reversed and converted with SWAR
SDX_DEV int lane_hex(const LaneBits& B, int a, int e, uint8_t* dst) {
  const int nb = e - a;
  if (nb <= 0) return 0;
  const int nd = (nb + 3) >> 2;
  if (!dst) return nd;
  for (int c = 0; c < nd; c += 8) {
    const int cnt = nd - c < 8 ? nd - c : 8;
    const int s0 = e - 4 * (nd - c), s = s0 > a ? s0 : a;   // bits before a read as 0
    const uint32_t v = B.win(s, 4 * cnt - (s - s0));        // the chunk's value, right-aligned
    uint64_t x = (uint64_t)v << (64 - 4 * cnt);             // first digit in the top nibble
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);  // nibble reverse
    x = ((x >> 8) & 0x00FF00FF00FF00FFull) | ((x & 0x00FF00FF00FF00FFull) << 8);
    x = ((x >> 16) & 0x0000FFFF0000FFFFull) | ((x & 0x0000FFFF0000FFFFull) << 16);
    x = (x >> 32) | (x << 32);                              // digit i in nibble i (i < cnt)
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;            // 8 nibbles -> 8 bytes
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    const uint64_t ge10 = ((x + 0x0606060606060606ull) >> 4) & 0x0101010101010101ull;
    x += 0x3030303030303030ull + ge10 * 7ull;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < cnt) dst[c + i] = (uint8_t)(x >> (8 * i));
  }
  return nd;
}

// bin_str_2_hex_str(bits[a1:e1]) == bin_str_2_hex_str(bits[a2:e2]) (e >= a)
SDX_DEV bool hex_equal(const LaneBits& B, int a1, int e1, int a2, int e2) {
  if (((e1 - a1 + 3) >> 2) != ((e2 - a2 + 3) >> 2)) return false;
  const int m = (e1 - a1 > e2 - a2) ? e1 - a1 : e2 - a2;
  // right-aligned, 32 bits per step; bits left of a1 / a2 count as 0
  for (int t = 0; t < m; t += 32) {
    const int k = m - t < 32 ? m - t : 32;
    const int s1 = e1 - t - k, s2 = e2 - t - k;
    const int v1 = e1 - t - (s1 > a1 ? s1 : a1), v2 = e2 - t - (s2 > a2 ? s2 : a2);
    const uint32_t x = v1 > 0 ? B.win(e1 - t - v1, v1) : 0u;
    const uint32_t y = v2 > 0 ? B.win(e2 - t - v2, v2) : 0u;
    if (x != y) return false;
  }
  return true;
}

// length_in_range(protocol_id, n) (helpers.py:124-166): 0 = in range, else the failure text
// (1 'message is too short', 2 'message is too long', 3 'protocol does not exists')
SDX_DEV int mc_lir(const sdx_mc_proto* r, int n) {
  if (cld(&r->lir_noexist)) return 3;
  const int lo = cld(&r->has_lmin) ? cld(&r->lmin) : -1;
  if (lo != -1 && n < lo) return 1;
  if (cld(&r->has_lmax) && n > cld(&r->lmax)) return 2;
  return 0;
}

// slice bounds of bit_data[a:e] for a string of n bits
SDX_DEV int clip_end(int a, int e, int n) {
  const int x = e < n ? e : n;
  return x > a ? x : a;
}

// TFA message iterator (manchester.py:615-719): yields [pos, message_end) per do-while round;
// finds run over the n bits of the string, the loop bound and the not-found end are mcbitnum
struct TfaIter {
  int pos, end, n, mb, loops;
  SDX_DEV bool next(const LaneBits& B, int* a, int* e) {
    if (!(end < mb)) return false;
    int me = B.find(0x1FFDu /*1111111111101*/, 13, pos, n);
    if (me < pos) me = mb;
    *a = pos;
    *e = me;
    end = me;
    const int nx = B.find(0xDu /*1101*/, 4, me, n);
    if (nx != -1) pos = nx + 4;
    else end = mb;
    ++loops;
    return true;
  }
};

// result of one method call: rc and how to print it
struct McOut {
  int rc;        // 1 ok, 0 (-1, msg) with why, -1 raise TypeError, -2 raise ValueError
  int kind;      // 0 hex window, 1 funkbus bytes, 2 tfa list, 3 sainlogic padded window
  int a, e;      // hex window
  uint64_t fb;   // funkbus 6 bytes (big-endian)
  int len;       // payload length without the preamble
  int why;       // enum McWhy when rc == 0
  int aux;       // MCW_TFA_NODUP: retmsg; MCW_SOMFY: len(bit_data)
};

SDX_DEV McOut mc_fail(int why, int aux = 0) { return McOut{0, 0, 0, 0, 0, 0, why, aux}; }

// the TFA duplicate scan shared by the length pass (dst == nullptr) and the writer
SDX_DEV int tfa_scan(const sdx_mc_proto* r, const LaneBits& B, int n, int mb, int p0, uint8_t* dst, int* last_fail,
                     int* loops) {
  TfaIter it{p0, -1, n, mb, 1}, outer = it;
  int a, e, j = 0, q = 0, nd = 0;
  if (dst) dst[q] = '[';
  ++q;
  while (outer.next(B, &a, &e)) {
    const int f = mc_lir(r, e - a);
    if (f == 0) {
      const int ec = clip_end(a, e, n);
      int eq = 0, a2, e2, k = 0;
      TfaIter inner = it;
      while (k < j && inner.next(B, &a2, &e2)) {
        if (mc_lir(r, e2 - a2) == 0 && hex_equal(B, a, ec, a2, clip_end(a2, e2, n))) ++eq;
        ++k;
      }
      if (eq == 1) {  // seen exactly once before: a duplicate
        if (nd) {
          if (dst) { dst[q] = ','; dst[q + 1] = ' '; }
          q += 2;
        }
        if (dst) dst[q] = '\'';
        ++q;
        q += lane_hex(B, a, ec, dst ? dst + q : nullptr);
        if (dst) dst[q] = '\'';
        ++q;
        ++nd;
      }
    } else if (last_fail) {
      *last_fail = f;
    }
    ++j;
  }
  if (dst) dst[q] = ']';
  ++q;
  if (loops) *loops = outer.loops;
  return nd ? q : 0;
}

// one MC method on bits B[0, n) with mcbitnum mb (D: the mc2dmc view of B for Funkbus).
// `method` is the record's method (enum sdx_mc_method); the unit entry may override it.
SDX_DEV McOut mc_method(const sdx_mc_proto* r, int method, const LaneBits& B, int n, int mb, const LaneBits& D) {
  McOut o{0, 0, 0, 0, 0, 0, 0, 0};
  switch (method) {
    case SDX_MC_FUNKBUS: {  // manchester.py:207-300
      const int lmin = cld(&r->has_lmin) ? cld(&r->lmin) : -1;
      if (mb < lmin) return mc_fail(MCW_SHORT);
      if (cld(&r->has_lmax) && mb > cld(&r->lmax)) return mc_fail(MCW_LONG);
      const int pidn = cld(&r->pid_num);
      if (pidn == SDX_PID_NOT_INT) { o.rc = -2; return o; }  // int(protocol_id) raises
      const int dn = n > 0 ? n - 1 : 0;  // mc2dmc of the lh/hl expansion
      int base, slen;
      if (pidn == 119) {
        const int pos = D.find(0xCu /*01100*/, 5, 0, dn);
        if (!(pos >= 0 && pos < 5)) return mc_fail(MCW_BEGIN);
        base = pos;
        slen = 3 + dn - pos;
        if (slen < 48) return mc_fail(MCW_BEGIN);
      } else {
        base = 0;
        slen = 1 + dn;
      }
      const uint32_t pre = (pidn == 119) ? 1u /*001*/ : 0u;
      const int plen = (pidn == 119) ? 3 : 1;
      auto sbit = [&](int t) -> int { return t < plen ? (int)((pre >> (plen - 1 - t)) & 1) : D.get(base + t - plen); };
      uint64_t bytes = 0;
      int xr = 0, chk = 0, par = 0;
      for (int i = 0; i < 6; ++i) {
        const int a = 8 * i, e = (8 * i + 8 < slen) ? 8 * i + 8 : slen;
        if (e <= a) { o.rc = -2; return o; }  // int('', 2)
        int d = 0;
        for (int t = a; t < e; ++t) d = (d << 1) | sbit(t);
        bytes = (bytes << 8) | (uint64_t)d;
        if (i < 5) xr ^= d;
        else {
          chk = d & 0x0F;
          xr ^= d & 0xE0;
          d &= 0xF0;
        }
        par ^= __popc(d) & 1;
      }
      if (par == 1) return mc_fail(MCW_PARITY);
      const int nib = ((xr & 0xF0) >> 4) ^ (xr & 0x0F);
      int res = 0;
      if (nib & 8) res ^= 0xC;
      if (nib & 4) res ^= 0x2;
      if (nib & 2) res ^= 0x8;
      if (nib & 1) res ^= 0x3;
      if (res != chk) return mc_fail(MCW_CHECKSUM);
      o.rc = 1; o.kind = 1; o.fb = bytes; o.len = 12;
      return o;
    }
    case SDX_MC_SAINLOGIC: {  // manchester.py:302-354
      const int lmax = cld(&r->has_lmax) ? cld(&r->lmax) : 0;
      if (mb > lmax) return mc_fail(MCW_LONG);
      int pad = 0, m = n, mbn = mb;
      if (mb < 128) {
        const int st = B.find(0x14u /*010100*/, 6, 0, n);
        if (st < 0 || st > 10) return mc_fail(MCW_SAIN_START);
        pad = st < 10 ? 10 - st : 0;  // '1' prepended until the sync sits at 10
        m = (n + pad < 128) ? n + pad : 128;
        mbn = m;
      }
      const int lmin = cld(&r->has_lmin) ? cld(&r->lmin) : 0;
      if (mbn < lmin) return mc_fail(MCW_SHORT);
      // bits = '1'*pad + B[0 : m-pad]; encode as window with a virtual prefix
      o.rc = 1; o.kind = 3; o.a = pad; o.e = m; o.len = (m + 3) >> 2;
      return o;
    }
    case SDX_MC_AS: {  // manchester.py:356-416
      const int lmin = cld(&r->has_lmin) ? cld(&r->lmin) : -1, lmax = cld(&r->has_lmax) ? cld(&r->lmax) : 9999;
      const int st = B.find(0xCu /*1100*/, 4, 16, n);
      if (st >= 0) {
        int en = B.find(0xCu, 4, st + 16, n);
        if (en == -1) en = n;
        const int ml = en - st;
        if (ml < lmin) return mc_fail(MCW_SHORT);
        if (ml > lmax) return mc_fail(MCW_LONG);
        o.rc = 1; o.a = st; o.e = n; o.len = (n - st + 3) >> 2;
        return o;
      }
      if (mb < lmin) return mc_fail(MCW_SHORT);
      if (mb > lmax) return mc_fail(MCW_LONG);
      o.rc = 1; o.a = 0; o.e = n; o.len = (n + 3) >> 2;
      return o;
    }
    case SDX_MC_PLAIN: {  // manchester.py:418-586 (Hideki, Maverick, OSV1, OSV2o3, OSPIR)
      const int lmin = cld(&r->has_lmin) ? cld(&r->lmin) : -1, lmax = cld(&r->has_lmax) ? cld(&r->lmax) : 9999;
      if (mb < lmin) return mc_fail(MCW_SHORT);
      if (mb > lmax) return mc_fail(MCW_LONG);
      o.rc = 1; o.a = 0; o.e = n; o.len = (n + 3) >> 2;
      return o;
    }
    case SDX_MC_RAW: {  // manchester.py:588-613
      const int lmax = cld(&r->has_lmax) ? cld(&r->lmax) : 0;
      if (mb > lmax) return mc_fail(MCW_LONG);
      o.rc = 1; o.a = 0; o.e = n; o.len = (n + 3) >> 2;
      return o;
    }
    case SDX_MC_HMCRAW: {  // helpers.py:90-122: un-converted str length_max -> int > str TypeError
      if (cld(&r->has_lmax)) {
        if (cld(&r->lmax_is_str)) { o.rc = -1; return o; }
        if (mb > cld(&r->lmax)) return mc_fail(MCW_TO_LONG);
      }
      o.rc = 1; o.a = 0; o.e = n; o.len = (n + 3) >> 2;
      return o;
    }
    case SDX_MC_TFA: {  // manchester.py:615-719
      const int p0 = B.find(0xFFDu /*111111111101*/, 12, 0, n);
      if (p0 == -1) return mc_fail(MCW_TFA_SYNC);
      int last_fail = 0, loops = 0;
      const int len = tfa_scan(r, B, n, mb, p0 + 12, nullptr, &last_fail, &loops);
      if (loops == 10) return mc_fail(MCW_TFA_LOOP);
      if (len == 0) return mc_fail(MCW_TFA_NODUP, last_fail);
      o.rc = 1; o.kind = 2; o.len = len; o.a = p0 + 12;
      return o;
    }
    case SDX_MC_GROTHE: {  // manchester.py:721-754
      if (mb != 32) return mc_fail(MCW_GROTHE);
      o.rc = 1; o.a = 0; o.e = n; o.len = (n + 3) >> 2;
      return o;
    }
    case SDX_MC_SOMFY: {  // manchester.py:756-795
      int a = 0, e = n;
      if (mb == 57) { a = n > 0 ? 1 : 0; e = n < 57 ? n : 57; if (e < a) e = a; }  // bit_data[1:57]
      if (e - a != 56) return mc_fail(MCW_SOMFY, e - a);
      o.rc = 1; o.a = a; o.e = e; o.len = 14;
      return o;
    }
  }
  return o;
}

SDX_DEV void mc_write(const sdx_mc_proto* r, const McOut& o, const LaneBits& B, int n, int mb, uint8_t* dst) {
  if (o.kind == 0) {
    lane_hex(B, o.a, o.e, dst);
  } else if (o.kind == 1) {
    for (int i = 0; i < 12; ++i) {
      const int v = (int)((o.fb >> (4 * (11 - i))) & 15);
      dst[i] = (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10);
    }
  } else if (o.kind == 3) {  // Sainlogic: '1'*pad + bits, truncated to e characters
    const int pad = o.a, m = o.e, nd = (m + 3) >> 2;
    for (int d = 0; d < nd; ++d) {
      const int de = m - 4 * (nd - 1 - d), da = (de - 4 > 0) ? de - 4 : 0;
      int v = 0;
      for (int i = da; i < de; ++i) v = (v << 1) | (i < pad ? 1 : B.get(i - pad));
      dst[d] = (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10);
    }
  } else {  // TFA: Python list repr "['A', 'B']"
    tfa_scan(r, B, n, mb, o.a, dst, nullptr, nullptr);
  }
}

}  // namespace sdx
