// sdx_lines.hip -- the wire-line front end, hand-written HIP for gfx950.
//
// Raw firmware lines -> demodulator batches, one lane per line, entirely on the device.  Per line
// this restates what the reference does before demodulation:
//   transport.py:123            bytes.decode("latin-1").strip()  (bytes here = the latin-1 string)
//   parser/__init__.py:37-49    SignalParser.parse_line: extract_payload, route by payload[:2].upper()
//   parser/base.py:188-206      extract_payload: strip, ^\x02(M[sSuUcCNOo];.*;)\x03$
//   parser/base.py:13-186       decompress_payload (Mred=1 lines)
//   parser/mu.py:48-68          the MU validity regex, _parse_to_dict, "D" required
//   parser/ms.py:35-41          _parse_to_dict, "D" required
//   parser/mc.py:37-155         MC header validation, required D/C/L, hex D, int(R)/int(F)
//   parser/mn.py:17,31-51       MN_PATTERN (the hex characters become an sdx_mn_batch frame)
//   sd_protocols/message_*.py   the P#/CP/SP/R/data string gates the demodulators apply
// The outputs of line i are message i of an sdx_pulse_batch / sdx_mc_batch in slot layout
// (len_dev), so the demodulation kernels read them in place.  Anything whose exact Python meaning
// this file does not model (bytes >= 0x80 after decompression, multi-digit pattern ids, non-integer
// pattern values) is reported SDX_LS_UNSUPPORTED instead of being approximated.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/sdx.h"

namespace sdx {
int set_error(int code, const std::string& msg);  // sdx_kernels.hip
}

namespace sdxl {

#define LD __device__ __forceinline__

#ifdef SDX_LPROF  // k_parse_comp phase profile (variant builds only): per-lane s_memtime deltas
__device__ unsigned long long g_lprof[16];
#define LP_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define LP_ADD(slot, t0) lp[slot] += __builtin_amdgcn_s_memtime() - (t0)
#define LP_ARG , unsigned long long* lp
#define LP_PASS , lp
#else
#define LP_T(v)
#define LP_ADD(slot, t0)
#define LP_ARG
#define LP_PASS
#endif

struct Str {
  const uint8_t* p;
  int n;
};

// Python character classes on a latin-1 character (tables checked in tests/test_lines.py)
LD bool py_space(uint8_t c) { return (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x20) || c == 0x85 || c == 0xa0; }
LD bool digit(uint8_t c) { return c >= '0' && c <= '9'; }
LD bool hexc(uint8_t c) { return digit(c) || ((c | 32) >= 'a' && (c | 32) <= 'f'); }
LD bool py_alpha(uint8_t c) {
  if ((c | 32) >= 'a' && (c | 32) <= 'z') return true;
  return c == 0xaa || c == 0xb5 || c == 0xba || (c >= 0xc0 && c <= 0xd6) || (c >= 0xd8 && c <= 0xf6) || c >= 0xf8;
}
LD bool py_alnum_ascii(uint8_t c) { return c < 128 && (digit(c) || ((c | 32) >= 'a' && (c | 32) <= 'z')); }
LD uint8_t up(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }
LD int hexv(uint8_t c) { return digit(c) ? c - '0' : ((c | 32) - 'a' + 10); }

// appends bytes to global memory, one 8-byte store per aligned word; the first and the last
// (partial) words are written byte by byte, so no byte outside [d, d + n) is touched
struct Writer8 {
  uint8_t* w;    // aligned word being filled
  int n, cap;
  bool ovf;
  uint64_t acc;
  int fill;      // bytes of the word filled (incl. the skipped head)
  int head;      // bytes of the first word before d
  LD Writer8(uint8_t* dst, int capacity)
      : w(dst - ((uintptr_t)dst & 7)), n(0), cap(capacity), ovf(false), acc(0), fill((int)((uintptr_t)dst & 7)),
        head((int)((uintptr_t)dst & 7)) {}
  LD void flush() {
    if (head) {
      for (int k = head; k < 8; ++k) w[k] = (uint8_t)(acc >> (8 * k));
      head = 0;
    } else {
      *reinterpret_cast<uint64_t*>(w) = acc;
    }
    w += 8;
    acc = 0;
    fill = 0;
  }
  LD void put(uint8_t c) {
    if (n >= cap) {
      ovf = true;
      ++n;
      return;
    }
    acc |= (uint64_t)c << (8 * fill);
    ++n;
    if (++fill == 8) flush();
  }
  LD void put_uint(uint32_t v) {
    char t[10];
    int k = 0;
    do {
      t[k++] = (char)('0' + v % 10);
      v /= 10;
    } while (v);
    while (k) put((uint8_t)t[--k]);
  }
  // 8 characters (x's bytes, lowest first): one aligned 8-byte store, the characters that spill
  // into the next word stay in acc
  LD void put8(uint64_t x) {
    if (head || n + 8 > cap) {
      for (int t = 0; t < 8; ++t) put((uint8_t)(x >> (8 * t)));
      return;
    }
    n += 8;
    if (fill == 0) {
      *reinterpret_cast<uint64_t*>(w) = x;
    } else {
      *reinterpret_cast<uint64_t*>(w) = acc | (x << (8 * fill));
      acc = x >> (64 - 8 * fill);
    }
    w += 8;
  }
  LD void finish() {
    for (int k = head; k < fill; ++k) w[k] = (uint8_t)(acc >> (8 * k));
    fill = head = 0;
  }
  LD void mark_d(bool) {}
};

// appends bytes to a lane's LDS buffer: one byte store per character, no word assembly (the
// assembling Writer8's flush branch diverges across a wave's lanes on almost every character)
struct LdsWriter {
  uint8_t* p;
  int n, cap;
  bool ovf;
  LD LdsWriter(uint8_t* dst, int capacity) : p(dst), n(0), cap(capacity), ovf(false) {}
  LD void put(uint8_t c) {
    if (n < cap) p[n] = c;
    else ovf = true;
    ++n;
  }
  LD void put_uint(uint32_t v) {
    char t[10];
    int k = 0;
    do {
      t[k++] = (char)('0' + v % 10);
      v /= 10;
    } while (v);
    while (k) put((uint8_t)t[--k]);
  }
  LD void put8(uint64_t x) {
    for (int t = 0; t < 8; ++t) put((uint8_t)(x >> (8 * t)));
  }
  LD void finish() {}
  LD void mark_d(bool) {}
};

// the first ';' at or after s, or P.n: aligned 8-byte words, SWAR ';' test (no byte at or after
// P.n counts; the words read are the ones holding bytes of [s, P.n))
LD int find_semi(const Str& P, int s) {
  if (s >= P.n) return P.n;
  const uint8_t* q = P.p + s;
  const int al = (int)((uintptr_t)q & 7);
  const uint64_t* w = reinterpret_cast<const uint64_t*>(q - al);
  int base = s - al;
  uint64_t x = *w;
  uint64_t valid = ~0ull << (8 * al);  // bytes of the first word before s do not count
  while (true) {
    const uint64_t t = x ^ 0x3B3B3B3B3B3B3B3Bull;
    uint64_t z = ~(((t & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | t) & 0x8080808080808080ull;
    z &= valid;
    const int left = P.n - base;  // bytes of this word inside P (> 0)
    if (left < 8) z &= ~0ull >> (64 - 8 * left);
    if (z) return base + (__builtin_ctzll(z) >> 3);
    if (left <= 8) return P.n;
    base += 8;
    x = *++w;
    valid = ~0ull;
  }
}

// next non-empty ';'-separated part at or after pos: [s, e); returns false at the end
LD bool next_part(const Str& P, int& pos, int& s, int& e) {
  while (pos <= P.n) {
    s = pos;
#ifdef SDX_NEXTPART_BYTES
    e = s;
    while (e < P.n && P.p[e] != ';') ++e;
#else
    e = find_semi(P, s);
#endif
    pos = e + 1;
    if (e > s) return true;
  }
  return false;
}

// base.py:76-99: does this part end the merged D= payload?
LD bool d_field(const Str& P, int s, int e) {
  const uint8_t m0 = P.p[s];
  const int m1n = e - s - 1;
  if (!py_alpha(m0)) return false;
  if (m0 == 'D' || m0 == 'd') return true;
  if (m0 > 127) return true;
  if (m0 == 'M') return true;
  if ((m0 == 'C' || m0 == 'S') && m1n == 1) return true;
  if (m0 == 'o' || m0 == 'm') return true;
  if (m1n >= 1 && m1n <= 2 && hexc(P.p[s + 1]) && (m1n == 1 || hexc(P.p[s + 2]))) return true;
  for (int i = s; i < e; ++i)
    if (P.p[i] == '=') return true;  // alnum (ASCII letter here) and '=' in the part
  return false;
}

// decompress_payload (base.py:13-186) into w; returns false when an upper() of a non-ASCII
// character would be needed (UNSUPPORTED)
// one non-D part of decompress_payload (base.py:142-181); false: str.upper() of a non-ASCII byte
template <class W>
LD bool dec_part(const Str& P, int s, int e, W& w) {
  const uint8_t m0 = P.p[s];
  const int m1s = s + 1, m1n = e - s - 1;
  if (m0 == 'M') {  // :144-146
    w.put('M');
    for (int i = m1s; i < e; ++i) {
      if (P.p[i] >= 128) return false;
      w.put(up(P.p[i]));
    }
  } else if (m0 > 127) {  // :149-165
    w.put('P');
    w.put((uint8_t)('0' + (m0 & 7)));
    w.put('=');
    if (m1n == 2) {
      uint32_t ml = P.p[m1s] & 127, mh = P.p[m1s + 1] & 127;
      if (m0 & 32) w.put('-');
      if (m0 & 16) ml += 128;
      w.put_uint(mh * 256 + ml);
    }
  } else if ((m0 == 'C' || m0 == 'S') && m1n == 1) {  // :168-169
    w.put(m0);
    w.put('P');
    w.put('=');
    w.put(P.p[m1s]);
  } else if (m0 == 'o' || m0 == 'm') {  // :172-173
    for (int i = s; i < e; ++i) w.put(P.p[i]);
  } else if (m1n >= 1 && m1n <= 2 && hexc(P.p[m1s]) && (m1n == 1 || hexc(P.p[m1s + 1]))) {  // :176-177
    w.put(m0);
    w.put('=');
    w.put_uint(m1n == 1 ? hexv(P.p[m1s]) : 16 * hexv(P.p[m1s]) + hexv(P.p[m1s + 1]));
  } else {  // :180-181 (ASCII alnum)
    w.put(m0);
    if (m1n) w.put('=');
    for (int i = m1s; i < e; ++i) w.put(P.p[i]);
  }
  return true;
}

// does decompress_payload emit anything for this part (the branches of :59-181)
LD bool dec_emits(const Str& P, int s, int e) {
  const uint8_t m0 = P.p[s];
  const int m1n = e - s - 1;
  return m0 == 'D' || m0 == 'd' || m0 == 'M' || m0 > 127 || ((m0 == 'C' || m0 == 'S') && m1n == 1) || m0 == 'o' ||
         m0 == 'm' || (m1n >= 1 && m1n <= 2 && hexc(P.p[s + 1]) && (m1n == 1 || hexc(P.p[s + 2]))) ||
         py_alnum_ascii(m0);
}

// a D/d part (:59-140) starting at part [s, e); pos = where the part loop resumes
// four data bytes c (all < 0x80) -> the eight characters '0' + (c >> 4), '0' + (c & 7), in order
LD uint64_t expand_word(uint32_t v) {
  uint64_t y = v;
  y = (y | (y << 16)) & 0x0000FFFF0000FFFFull;
  y = (y | (y << 8)) & 0x00FF00FF00FF00FFull;  // byte t -> the low byte of 16-bit lane t
  return ((y >> 4) & 0x000F000F000F000Full) | ((y & 0x0007000700070007ull) << 8) | 0x3030303030303030ull;
}

template <class W>
LD void dec_data(const Str& P, int s, int e, int& pos, W& w) {
  const uint8_t m0 = P.p[s];
  const int m1s = s + 1;
  w.put('D');
  w.put('=');
  w.mark_d(true);
  // extent: the first part plus the following parts that do not start a field
  int lastend = e, j = pos, s2, e2;
  while (true) {
    const int before = j;
    if (!next_part(P, j, s2, e2)) {
      pos = j;
      break;
    }
    if (d_field(P, s2, e2)) {
      pos = before;  // the loop resumes at this part
      break;
    }
    lastend = e2;
    pos = j;
  }
  // f"{(c >> 4) & 15}{c & 7}" for every byte of m1 + (';' + part)*, runs of ';' collapsed (the empty
  // parts in between are dropped); 'd' drops the last digit (:130-131), then a leading '8' is
  // dropped (:134-135) -- both applied while streaming.  Bytes are read eight at a time.
  bool firstc = true;
  uint8_t prev = 0;
  const uint8_t* q = P.p + m1s;
  const int al = (int)((uintptr_t)q & 7);
  const uint64_t* wp = reinterpret_cast<const uint64_t*>(q - al);
  for (int k0 = m1s - al; k0 < lastend; k0 += 8) {
    const uint64_t x = *wp++;
    // a whole word inside the value, past its first character, not the last one of a 'd' part,
    // no byte >= 0x80 and no ';': two characters per byte, '0' + (c >> 4) and '0' + (c & 7)
    const uint64_t ts = x ^ 0x3B3B3B3B3B3B3B3Bull;
    const uint64_t semi = ~(((ts & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | ts) & 0x8080808080808080ull;
    if (!firstc && k0 >= m1s && k0 + 8 <= lastend && !(m0 == 'd' && k0 + 8 == lastend) &&
        ((x & 0x8080808080808080ull) | semi) == 0) {
      w.put8(expand_word((uint32_t)x));
      w.put8(expand_word((uint32_t)(x >> 32)));
      prev = (uint8_t)(x >> 56);
      continue;
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int k = k0 + b;
      if (k < m1s || k >= lastend) continue;
      const uint8_t c = (uint8_t)(x >> (8 * b));
      const bool skip = c == ';' && k > m1s && prev == ';';
      prev = c;
      if (skip) continue;
      const uint8_t h = (c >> 4) & 0xF;
      uint8_t c1 = h >= 10 ? '1' : (uint8_t)('0' + h);
      if (firstc) {
        firstc = false;
        if (c1 == '8') c1 = 0;  // the leading '8'
      }
      if (c1) w.put(c1);
      if (h >= 10) w.put((uint8_t)('0' + h - 10));
      if (!(m0 == 'd' && k == lastend - 1)) w.put((uint8_t)('0' + (c & 0x7)));
    }
  }
  w.mark_d(false);
}

// decompress_payload (base.py:13-186) of a payload that has a byte > 127 after its header.  The
// parts before the first D/d part, that part, and the rest are three loops, so that the lanes of
// a wave expand their (long) data parts together.
template <class W>
LD bool decompress(const Str& P, W& w) {
  int pos = 0, s = 0, e = 0;
  bool first = true, dpart = false;
  while (next_part(P, pos, s, e)) {  // parts before the data
    if (P.p[s] == 'D' || P.p[s] == 'd') {
      dpart = true;
      break;
    }
    if (!dec_emits(P, s, e)) continue;
    if (!first) w.put(';');
    first = false;
    if (!dec_part(P, s, e, w)) return false;
  }
  if (dpart) {
    if (!first) w.put(';');
    first = false;
    dec_data(P, s, e, pos, w);
    while (next_part(P, pos, s, e)) {  // the rest (a second data part is possible)
      if (!dec_emits(P, s, e)) continue;
      w.put(';');
      if (P.p[s] == 'D' || P.p[s] == 'd') dec_data(P, s, e, pos, w);
      else if (!dec_part(P, s, e, w)) return false;
    }
  }
  w.put(';');  // :184
  w.finish();
  return true;
}

LD bool lit(const Str& P, int pos, const char* s) {
  for (int i = 0; s[i]; ++i)
    if (pos + i >= P.n || P.p[pos + i] != (uint8_t)s[i]) return false;
  return true;
}
LD int digits_at(const Str& P, int pos) {
  int k = 0;
  while (pos + k < P.n && digit(P.p[pos + k])) ++k;
  return k;
}

// parser/mu.py:48 ^(?=.*D=\d+)(?:MU;(?:P[0-7]=-?[0-9]{1,5};){2,8}((?:D=\d{2,};)|(?:CP=\d;)|(?:R=\d+;)|
// (?:O;)|(?:e;)|(?:p;)|(?:w=\d;))*)$  -- no item can start like another, so one left-to-right scan
// decides it (and with a D item present the lookahead holds)
LD bool mu_valid(const Str& P) {
  int n = P.n;
  if (n > 0 && P.p[n - 1] == '\n') --n;  // '$' also matches before a final newline
  Str Q{P.p, n};
  if (!lit(Q, 0, "MU;")) return false;
  int pos = 3, np = 0;
  while (pos < n && Q.p[pos] == 'P') {
    if (np == 8) return false;  // a ninth P item cannot match anything
    if (pos + 2 >= n || Q.p[pos + 1] < '0' || Q.p[pos + 1] > '7' || Q.p[pos + 2] != '=') return false;
    int q = pos + 3;
    if (q < n && Q.p[q] == '-') ++q;
    const int k = digits_at(Q, q);
    if (k < 1 || k > 5 || q + k >= n || Q.p[q + k] != ';') return false;
    pos = q + k + 1;
    ++np;
  }
  if (np < 2) return false;
  bool hasd = false;
  while (pos < n) {
    const uint8_t c = Q.p[pos];
    if (c == 'D' && lit(Q, pos, "D=")) {
      const int k = digits_at(Q, pos + 2);
      if (k < 2 || pos + 2 + k >= n || Q.p[pos + 2 + k] != ';') return false;
      pos += 3 + k;
      hasd = true;
    } else if (c == 'C' && lit(Q, pos, "CP=")) {
      if (pos + 4 >= n || !digit(Q.p[pos + 3]) || Q.p[pos + 4] != ';') return false;
      pos += 5;
    } else if (c == 'R' && lit(Q, pos, "R=")) {
      const int k = digits_at(Q, pos + 2);
      if (k < 1 || pos + 2 + k >= n || Q.p[pos + 2 + k] != ';') return false;
      pos += 3 + k;
    } else if ((c == 'O' || c == 'e' || c == 'p') && pos + 1 < n && Q.p[pos + 1] == ';') {
      pos += 2;
    } else if (c == 'w' && lit(Q, pos, "w=")) {
      if (pos + 3 >= n || !digit(Q.p[pos + 2]) || Q.p[pos + 3] != ';') return false;
      pos += 4;
    } else {
      return false;
    }
  }
  return hasd;
}

// Python float(str) (float_from_string): ASCII whitespace stripped, '_' only between two digits,
// [+-]? (digits [. digits] | . digits) ([eE] [+-]? digits)?  or  [+-]? (inf | infinity | nan).
// 0 = ValueError (the reference's _patterns skips the key), 1 = *v exact, 2 = a valid float outside
// the modelled subset (SDX_LS_UNSUPPORTED).  Exact subset (Clinger's fast path): the significant
// digits form M < 2^53 (at most 19 of them, trailing zeros moved into the exponent) and
// |exp10| <= 22, so M * 10^exp10 (or M / 10^-exp10) is ONE IEEE operation on exact operands,
// i.e. the correctly rounded value Python's strtod returns; zero keeps its sign; inf / nan.
__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
// float() strips ' ' and \t\n\v\f\r (not \x1c-\x1f, which str.isspace() counts; non-ASCII never gets here)
LD bool float_ws(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }
LD bool lower_is(const Str& P, int s, const char* w, int n) {
  for (int k = 0; k < n; ++k) {
    uint8_t c = P.p[s + k];
    if (c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
    if (c != (uint8_t)w[k]) return false;
  }
  return true;
}
LD int parse_pyfloat(const Str& P, int s, int e, double* v) {
  while (s < e && float_ws(P.p[s])) ++s;
  while (e > s && float_ws(P.p[e - 1])) --e;
  if (s == e) return 0;
  for (int i = s; i < e; ++i)  // _Py_string_to_number_with_underscores: digit '_' digit only
    if (P.p[i] == '_' && (i == s || i + 1 >= e || !digit(P.p[i - 1]) || !digit(P.p[i + 1]))) return 0;
  int i = s;
  bool neg = false;
  if (P.p[i] == '-' || P.p[i] == '+') {
    neg = P.p[i] == '-';
    ++i;
  }
  const int rem = e - i;
  if ((rem == 3 && lower_is(P, i, "inf", 3)) || (rem == 8 && lower_is(P, i, "infinity", 8))) {
    *v = neg ? -__builtin_inf() : __builtin_inf();
    return 1;
  }
  if (rem == 3 && lower_is(P, i, "nan", 3)) {  // CPython: -nan keeps its sign bit
    *v = __longlong_as_double(neg ? (long long)0xFFF8000000000000ull : 0x7FF8000000000000ll);
    return 1;
  }
  uint64_t M = 0;
  int sig = 0, e10 = 0;
  bool anyd = false, lost = false;
  auto take = [&](int d, bool frac) {
    anyd = true;
    if (M == 0 && d == 0) {
      if (frac) --e10;
      return;
    }
    if (sig < 19) {
      M = 10 * M + (uint64_t)d;
      ++sig;
      if (frac) --e10;
    } else {
      if (d) lost = true;  // a 20th significant digit: outside the exact subset
      if (!frac) ++e10;
    }
  };
  for (; i < e && (digit(P.p[i]) || P.p[i] == '_'); ++i)
    if (P.p[i] != '_') take(P.p[i] - '0', false);
  if (i < e && P.p[i] == '.') {
    ++i;
    for (; i < e && (digit(P.p[i]) || P.p[i] == '_'); ++i)
      if (P.p[i] != '_') take(P.p[i] - '0', true);
  }
  if (!anyd) return 0;
  if (i < e && (P.p[i] == 'e' || P.p[i] == 'E')) {
    int j = i + 1;
    bool eneg = false;
    if (j < e && (P.p[j] == '+' || P.p[j] == '-')) {
      eneg = P.p[j] == '-';
      ++j;
    }
    if (j < e && digit(P.p[j])) {  // otherwise the number ends before the 'e': trailing junk
      long long x = 0;
      for (; j < e && (digit(P.p[j]) || P.p[j] == '_'); ++j)
        if (P.p[j] != '_' && x < 100000) x = 10 * x + (P.p[j] - '0');
      e10 += (int)(eneg ? -x : x);
      i = j;
    }
  }
  if (i != e) return 0;
  if (M == 0) {
    *v = neg ? -0.0 : 0.0;
    return 1;
  }
  if (lost) return 2;
  while (M % 10 == 0) {
    M /= 10;
    ++e10;
  }
  if (M >= (1ull << 53) || e10 < -22 || e10 > 22) return 2;
  const double x = e10 >= 0 ? (double)M * kPow10[e10] : (double)M / kPow10[-e10];
  *v = neg ? -x : x;
  return 1;
}
// int() of [-+]?[0-9]+ (any length): 0 = empty, 1 = ok, 2 = not decimal, 3 = ok but |v| >= 2^31
LD int parse_dec(const Str& P, int s, int e, long long* v) {
  if (s == e) return 0;
  int i = s;
  bool neg = false;
  if (P.p[i] == '-' || P.p[i] == '+') {
    neg = P.p[i] == '-';
    ++i;
  }
  if (i == e) return 2;
  long long x = 0;
  bool big = false;
  for (; i < e; ++i) {
    if (!digit(P.p[i])) return 2;
    x = 10 * x + (P.p[i] - '0');
    if (x >= (1ll << 31)) {
      big = true;
      x = 1ll << 31;
    }
  }
  *v = neg ? -x : x;
  return big && !(neg && x == (1ll << 31)) ? 3 : 1;
}
LD bool all_digits(const Str& P, int s, int e) {
  if (s >= e) return false;
  for (int i = s; i < e; ++i)
    if (!digit(P.p[i])) return false;
  return true;
}
LD bool keq(const Str& P, int s, int e, const char* k) {
  int i = 0;
  for (; k[i]; ++i)
    if (s + i >= e || P.p[s + i] != (uint8_t)k[i]) return false;
  return s + i == e;
}

struct Field {
  int s, e;  // value range, s < 0: absent
};


// ---- the parse kernel -------------------------------------------------------------------------
// One lane per line, reading its line straight from HBM: byte loads for the few positional checks,
// aligned 8-byte loads with SWAR byte-class masks for every scan (framing, each field value).
// Compressed payloads are decompressed into the line's own slot region (its final place,
// RawFrame.line) and parsed there, by the same code.  Canonical payloads go through a one-pass
// fast path; everything else through parse_payload (the reference's dict semantics in full).
// The D characters of uncompressed lines are copied to the slot by the whole wave, one line at a
// time with consecutive bytes per store instruction.
constexpr int PT = 256;  // threads per workgroup

struct LineRes {
  uint8_t kind = SDX_LINE_NONE, status = SDX_LS_NOFRAME;
  int dS = 0, dE = 0;  // D (MU/MS) or hex (MC) characters in the payload
  Field fR{-1, -1}, fF{-1, -1};
};

LD int64_t shfl64(int64_t v, int src) {
  const int lo = __shfl((int)(uint32_t)v, src), hi = __shfl((int)(uint32_t)((uint64_t)v >> 32), src);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

LD bool same_key(const Str& P, int s1, int e1, int s2, int e2) {
  if (e1 - s1 != e2 - s2) return false;
  for (int k = 0; k < e1 - s1; ++k)
    if (P.p[s1 + k] != P.p[s2 + k]) return false;
  return true;
}

constexpr uint64_t SW_L1 = 0x0101010101010101ull, SW_H = 0x8080808080808080ull;
enum { CLS_DIGIT = 0, CLS_HEX = 1, CLS_ANY = 2 };

LD uint64_t sw_digits(uint64_t x) {  // high bit of each byte: '0'..'9'
  const uint64_t lo7 = x & ~SW_H;
  const uint64_t ge = ((lo7 | SW_H) - SW_L1 * 0x30) & SW_H;
  const uint64_t le = ((SW_L1 * 0x39 | SW_H) - lo7) & SW_H;
  return ge & le & ~x;
}
LD uint64_t sw_hexalpha(uint64_t x) {  // 'a'..'f' / 'A'..'F'
  const uint64_t lc = (x & ~SW_H) | (SW_L1 * 0x20);
  const uint64_t ge = ((lc | SW_H) - SW_L1 * 0x61) & SW_H;
  const uint64_t le = ((SW_L1 * 0x66 | SW_H) - lc) & SW_H;
  return ge & le & ~x;
}

// position of the first ';' at or after s, or -1 when a byte outside the class comes first
// (CLS_ANY: any ASCII byte).  P[0, n) must end with ';'.  The aligned 8-byte words are loaded
// SCAN_W at a time (independent loads: one memory round trip per SCAN_W words of a long field
// instead of one per word); a word holding no byte of [0, n) is not loaded.
#ifndef SDX_SCAN_W
#define SDX_SCAN_W 4
#endif
constexpr int SCAN_W = SDX_SCAN_W;
LD int scan_run(const uint8_t* P, int n, int s, int cls) {
  const uint8_t* q = P + s;
  const int a = (int)((uintptr_t)q & 7);
  const uint64_t* w = reinterpret_cast<const uint64_t*>(q - a);
  int base = s - a;
  uint64_t pre = a ? (~0ull >> (64 - 8 * a)) : 0ull;  // bytes before s: neutral '0'
  while (true) {
    uint64_t xs[SCAN_W];
#pragma unroll
    for (int k = 0; k < SCAN_W; ++k) xs[k] = base + 8 * k < n ? w[k] : SW_L1 * 0x3B;  // past P: ';' (never reached)
#pragma unroll
    for (int k = 0; k < SCAN_W; ++k) {
      uint64_t x = xs[k];
      if (k == 0) x = (x & ~pre) | (SW_L1 * 0x30 & pre);
      const uint64_t t = x ^ (SW_L1 * 0x3B);
      const uint64_t semi = (t - SW_L1) & ~t & SW_H;
      const uint64_t dg = sw_digits(x);
      const uint64_t tn = x ^ (SW_L1 * 0x0A);  // CLS_ANY: ASCII, not a newline
      const uint64_t nl = ((tn & ~SW_H) + ~SW_H | tn) & SW_H;  // high bit: byte != '\n'
      const uint64_t ok = cls == CLS_DIGIT ? dg : cls == CLS_HEX ? (dg | sw_hexalpha(x)) : (~x & nl & SW_H);
      const uint64_t bad = ~ok & SW_H;
      if (semi) {
        if (bad & ((semi & (0 - semi)) - 1)) return -1;  // a bad byte before the ';'
        return base + 8 * k + (__builtin_ctzll(semi) >> 3);
      }
      if (bad) return -1;
    }
    pre = 0;
    base += 8 * SCAN_W;
    w += SCAN_W;
  }
}

LD long long dec_value(const uint8_t* P, int s, int e) {
  long long v = 0;
  for (int k = s; k < e; ++k) v = 10 * v + (P[k] - '0');
  return v;
}

// ---- fast path: canonical firmware payloads ------------------------------------------------
// Sound but incomplete: it accepts only payloads in the firmware's canonical form -- per type a
// fixed key set, each key at most once (pattern ids single digit, values plain decimal), no
// non-ASCII bytes -- for which the reference's dict / gate semantics reduce to one left-to-right
// pass; anything else returns false and parse_payload decides.  Every part costs one scan_run (so
// the lanes of a wave share one loop whatever part they are in).
enum {
  KP = 1, KD, KCP, KSP, KR, KF, KC, KL, KLL, KLH, KSL, KSH, KM, KW, KIGN
};

LD bool fast_payload(const uint8_t* P, int n, LineRes& r, const sdx_lines_out& out, int i) {
  if (n < 4 || P[0] != 'M' || P[2] != ';' || P[n - 1] != ';') return false;
  const uint8_t t = P[1];
  const bool mu = t == 'U', ms = t == 'S', mc = t == 'C';
  if (!mu && !ms && !mc) return false;
  uint32_t have = 0, ids = 0;
  uint64_t idord = 0;
  int np = 0;
  int dS = 0, dE = 0, rS = -1, rE = -1, fS = -1, fE = -1, cpS = 0, cpE = 0;
  long long cval = 0, lval = 0;
  bool phase1 = false;  // MU: past the P items
  double* pval = out.pat_val_dev + 10 * (int64_t)i;
  uint8_t* pid = out.pat_id_dev + 10 * (int64_t)i;
  int s = 3;
  while (s < n) {
    const uint8_t b0 = P[s];
    if (b0 == ';') {  // an empty part: skipped by the parsers, a mismatch for the MU regex
      if (mu) return false;
      ++s;
      continue;
    }
    const uint8_t b1 = P[s + 1], b2 = s + 2 < n ? P[s + 2] : 0;
    // 1. the key, where its value starts, the value's byte class
    int key = 0, vs = s, cls = CLS_ANY;
    bool sign = false;
    if (b0 == 'P' && digit(b1) && b2 == '=') {
      key = KP, vs = s + 3, cls = CLS_DIGIT, sign = true;
    } else if (b1 == '=') {
      vs = s + 2;
      if (b0 == 'D') key = KD, cls = mc ? CLS_HEX : CLS_DIGIT;
      else if (b0 == 'R') key = KR, cls = CLS_DIGIT, sign = mc;
      else if (b0 == 'F') key = KF, cls = mc ? CLS_DIGIT : CLS_ANY, sign = mc;
      else if (mc && b0 == 'C') key = KC, cls = CLS_DIGIT;
      else if (mc && b0 == 'L') key = KL, cls = CLS_DIGIT;
      else if (mc && b0 == 'M') key = KM, cls = CLS_HEX, sign = true;
      else if (mu && b0 == 'w') key = KW, cls = CLS_DIGIT;
    } else if (b2 == '=') {
      vs = s + 3, cls = CLS_DIGIT;
      if (b0 == 'C' && b1 == 'P' && !mc) key = KCP;
      else if (b0 == 'S' && b1 == 'P' && ms) key = KSP;
      else if (mc && b0 == 'L' && (b1 == 'L' || b1 == 'H')) key = b1 == 'L' ? KLL : KLH, cls = CLS_HEX, sign = true;
      else if (mc && b0 == 'S' && (b1 == 'L' || b1 == 'H')) key = b1 == 'L' ? KSL : KSH, cls = CLS_HEX, sign = true;
    }
    if (!key) {  // a part no rule of this path names: MU O;/e;/p;, MS parts no gate reads
      if (mc) return false;
      if (ms && (b0 == 'P' || b0 == 'D' || b0 == 'C' || b0 == 'S' || b0 == 'R' || b0 == 'F')) return false;
      if (mu && !((b0 == 'O' || b0 == 'e' || b0 == 'p') && b1 == ';')) return false;
      key = KIGN, vs = s, cls = CLS_ANY;
    }
    int v0 = vs;
    bool neg = false;
    if (sign && (P[v0] == '-' || P[v0] == '+')) {
      if (P[v0] == '+' && key == KP) return false;  // float("+5"): left to parse_payload
      neg = P[v0] == '-';
      ++v0;
    }
    // 2. one scan for every kind of part
    const int e = scan_run(P, n, v0, cls);
    if (e < 0) return false;
    const int nv = e - v0;
    // 3. the key's rule
    const uint32_t bit = 1u << key;
    if (key != KP && key != KIGN && key != KW) {
      if (have & bit) return false;  // a repeated key: dict semantics left to parse_payload
      have |= bit;
    }
    if (mu && key != KP) {
      if (np < 2) return false;
      phase1 = true;
    }
    switch (key) {
      case KP: {
        if (mc || (mu && (phase1 || b1 > '7' || np == 8))) return false;
        const int id = b1 - '0';
        if (((ids >> id) & 1) || nv < 1 || nv > (mu ? 5 : 15)) return false;
        const double v = (double)dec_value(P, v0, e);
        pval[np] = neg ? -v : v;
        pid[np] = b1;
        ids |= 1u << id;
        idord |= (uint64_t)id << (4 * np);
        ++np;
        break;
      }
      case KD:
        if (nv < (mu ? 2 : 1)) return false;
        dS = v0, dE = e;
        break;
      case KCP:
        if (nv < 1 || nv > (mu ? 1 : 9)) return false;
        cpS = v0, cpE = e;
        break;
      case KSP:
      case KLL:
      case KLH:
      case KSL:
      case KSH:
      case KM:
        if (nv < 1) return false;
        break;
      case KR:
        if (nv < 1) return false;
        rS = vs, rE = e;
        break;
      case KF:
        if (mu || (mc && nv < 1)) return false;
        fS = vs, fE = e;
        break;
      case KC:
      case KL:
        if (nv < 1 || nv > 9) return false;
        (key == KC ? cval : lval) = dec_value(P, v0, e);
        break;
      case KW:
        if (nv != 1) return false;
        break;
      default:  // KIGN
        if (mu && e != s + 1) return false;
        break;
    }
    s = e + 1;
  }
  if (!(have & (1u << KD))) return false;
  if ((rS >= 0 && rE - rS > 15) || (fS >= 0 && fE - fS > 15)) return false;
  if (mc) {
    if ((have & ((1u << KC) | (1u << KL))) != ((1u << KC) | (1u << KL))) return false;
    out.clock_dev[i] = (int32_t)cval;
    out.mcbitnum_dev[i] = (int32_t)lval;
    out.mcflags_dev[i] = 0;
  } else {
    if (dE - dS > SDX_LONG_MAX) return false;
    if (ms) {
      if ((have & ((1u << KCP) | (1u << KSP))) != ((1u << KCP) | (1u << KSP))) return false;
      const long long cp = dec_value(P, cpS, cpE);
      int8_t slotv = -1;
      for (int z = 0; z < np; ++z)
        if (cp < 10 && (int)((idord >> (4 * z)) & 15) == cp) slotv = (int8_t)z;
      out.cp_slot_dev[i] = slotv;
      out.ms_ok_dev[i] = slotv >= 0 ? 1 : 0;
    }
    out.npat_dev[i] = (uint8_t)np;
  }
  r.kind = mu ? SDX_LINE_MU : ms ? SDX_LINE_MS : SDX_LINE_MC;
  r.status = SDX_LS_OK;
  r.dS = dS;
  r.dE = dE;
  r.fR = Field{rS, rE};
  r.fF = Field{fS, fE};
  return true;
}

// extract_payload (base.py:188-206) on the stripped line L[a, b): the positional checks, then one
// SWAR pass for '.' not matching a newline and for the bytes > 127 that make decompress_payload
// run (MS/MU/MO/MN).  Reads the aligned 8-byte words around the range.
LD bool frame_check(const uint8_t* L, int a, int b, bool& comp) {
  if (b - a < 6 || L[a] != 0x02 || L[b - 1] != 0x03 || L[a + 1] != 'M' || L[a + 3] != ';' || L[b - 2] != ';')
    return false;
  const uint8_t t = L[a + 2];
  if (!(t == 's' || t == 'S' || t == 'u' || t == 'U' || t == 'c' || t == 'C' || t == 'N' || t == 'O' || t == 'o'))
    return false;
  const int s = a + 4, e = b - 2;
  uint64_t acc = 0;
  if (s < e) {
    const uint8_t* q = L + s;
    const int al = (int)((uintptr_t)q & 7);
    const uint64_t* w = reinterpret_cast<const uint64_t*>(q - al);
    int rem = e - s + al;
    uint64_t m = al ? ~(~0ull >> (64 - 8 * al)) : ~0ull;
    for (; rem > 0; rem -= 8, ++w) {
      if (rem < 8) m &= ~0ull >> (64 - 8 * rem);
      const uint64_t x = *w & m;
      const uint64_t tt = x ^ (SW_L1 * 0x0A);
      if ((tt - SW_L1) & ~tt & SW_H) return false;
      acc |= x;
      m = ~0ull;
    }
  }
  const uint8_t t1 = up(t);
  comp = (acc & SW_H) && (t1 == 'S' || t1 == 'U' || t1 == 'O' || t1 == 'N');
  return true;
}

// MNParser.parse up to the protocol loop (parser/mn.py:33-51):
//   MN_PATTERN = ^MN;D=(Y?)([0-9A-F]+);(?:R=([0-9]+);)?(?:A=(-?[0-9]{1,3});)?$
// matched deterministically ('Y' is no hex digit; an optional group that starts but does not
// complete leaves text that '$' rejects).  '$' also matches before a final newline.
LD void mn_line(const Str& P, LineRes& r) {
  const uint8_t* p = P.p;
  const int n = P.n;
  r.status = SDX_LS_INVALID;
  if (n < 7 || p[0] != 'M' || p[1] != 'N' || p[2] != ';' || p[3] != 'D' || p[4] != '=') return;
  int k = 5;
  if (p[k] == 'Y') ++k;
  const int dS = k;
  while (k < n && (digit(p[k]) || (p[k] >= 'A' && p[k] <= 'F'))) ++k;
  if (k == dS || k >= n || p[k] != ';') return;
  const int dE = k++;
  Field fR{-1, -1}, fA{-1, -1};
  if (k + 1 < n && p[k] == 'R' && p[k + 1] == '=') {
    const int v = k + 2;
    int e = v;
    while (e < n && digit(p[e])) ++e;
    if (e == v || e >= n || p[e] != ';') return;
    fR = Field{v, e};
    k = e + 1;
  }
  if (k + 1 < n && p[k] == 'A' && p[k + 1] == '=') {
    const int v = k + 2;
    int e = v;
    if (e < n && p[e] == '-') ++e;
    const int ds = e;
    while (e < n && digit(p[e]) && e - ds < 3) ++e;
    if (e == ds || e >= n || p[e] != ';') return;
    fA = Field{v, e};
    k = e + 1;
  }
  if (!(k == n || (k == n - 1 && p[k] == '\n'))) return;
  if (dE - dS > SDX_MN_HEX_MAX || (fR.s >= 0 && fR.e - fR.s > 15)) {  // sdx_demod_mn / meta_dev contract
    r.status = SDX_LS_UNSUPPORTED;
    return;
  }
  r.status = SDX_LS_OK;
  r.dS = dS;
  r.dE = dE;
  r.fR = fR;
  r.fF = fA;  // A= travels in the F slot of meta_dev
}

// routing + the per-type parser rules on a (decompressed) payload; writes the pattern / MS / MC
// fields of line i, returns kind/status and the D/R/F ranges.  pvt = this lane's column of the
// fast P-key table (stride 64 words).
LD void parse_payload(const Str& P, LineRes& r, const sdx_lines_out& out, int i, uint32_t* pvt) {
  bool gen = false;  // MU/MS: a multi-digit pattern id or > SDX_LONG_MAX pulses (SDX_LS_GENERAL)
  // ---- routing: payload[:2].upper()
  const uint8_t c0 = P.n > 0 ? up(P.p[0]) : 0, c1 = P.n > 1 ? up(P.p[1]) : 0;
  if (c0 != 'M' || !(c1 == 'S' || c1 == 'U' || c1 == 'C' || c1 == 'N')) {
    r.status = SDX_LS_NOPARSER;
    return;
  }
  r.kind = c1 == 'U' ? SDX_LINE_MU : c1 == 'S' ? SDX_LINE_MS : c1 == 'C' ? SDX_LINE_MC : SDX_LINE_MN;
  if (r.kind == SDX_LINE_MN) {
    mn_line(P, r);
    return;
  }
  {
    uint8_t any = 0;
    for (int k = 0; k < P.n; ++k) any |= P.p[k];
    if (any & 0x80) {  // str methods on non-ASCII characters are not modelled
      r.status = SDX_LS_UNSUPPORTED;
      return;
    }
  }
  if (r.kind == SDX_LINE_MU && !mu_valid(P)) {
    r.status = SDX_LS_INVALID;
    return;
  }
  Field fD{-1, -1}, fCP{-1, -1}, fSP{-1, -1}, fC{-1, -1}, fL{-1, -1};
  Field& fR = r.fR;
  Field& fF = r.fF;
  if (r.kind == SDX_LINE_MC) {
    // ---- MCParser._parse_to_dict + key set + required fields (mc.py:37-56,95-139)
    int pos = 0, s, e;
    uint32_t seen = 0;  // LL LH SL SH D C L R F M MC Mc
    while (next_part(P, pos, s, e)) {
      int eq = -1;
      for (int k = s; k < e; ++k)
        if (P.p[k] == '=') {
          eq = k;
          break;
        }
      int bit = -1;
      if (eq >= 0) {
        const int kl = eq - s;
        bool keyok = kl >= 1 && kl <= 2;
        for (int k = s; k < eq && keyok; ++k) keyok = P.p[k] >= 'A' && P.p[k] <= 'Z';
        int v = eq + 1;
        if (v < e && (P.p[v] == '-' || P.p[v] == '+')) ++v;
        bool valok = v < e;
        for (int k = v; k < e && valok; ++k) valok = hexc(P.p[k]);
        if (!keyok || !valok) {
          r.status = SDX_LS_INVALID;
          return;
        }
        static const char* const KEYS[11] = {"LL", "LH", "SL", "SH", "D", "C", "L", "R", "F", "M", "MC"};
        for (int q = 0; q < 11 && bit < 0; ++q)
          if (keq(P, s, eq, KEYS[q])) bit = q;
        if (bit < 0) {  // a well-formed key outside the MC header set
          r.status = SDX_LS_INVALID;
          return;
        }
        const Field f{eq + 1, e};
        if (bit == 4) fD = f;
        if (bit == 5) fC = f;
        if (bit == 6) fL = f;
        if (bit == 7) fR = f;
        if (bit == 8) fF = f;
      } else {
        if (keq(P, s, e, "MC")) bit = 10;
        else if (keq(P, s, e, "Mc")) bit = 11;
        else {  // not MC/Mc: invalid after the first part, and outside the key set as the first
          r.status = SDX_LS_INVALID;
          return;
        }
      }
      if (seen & (1u << bit)) {  // duplicate key
        r.status = SDX_LS_INVALID;
        return;
      }
      seen |= 1u << bit;
    }
    if (fD.s < 0 || fC.s < 0 || fL.s < 0) {
      r.status = SDX_LS_INVALID;
      return;
    }
    for (int k = fD.s; k < fD.e; ++k)  // re.fullmatch(r"[0-9a-fA-F]+", raw_hex)
      if (!hexc(P.p[k])) {
        r.status = SDX_LS_INVALID;
        return;
      }
    long long v;
    const int rr = fR.s >= 0 ? parse_dec(P, fR.s, fR.e, &v) : 1, rf = fF.s >= 0 ? parse_dec(P, fF.s, fF.e, &v) : 1;
    if ((rr != 1 && rr != 3) || (rf != 1 && rf != 3)) {  // int(R) / int(F) raise -> ignored (mc.py:141-155)
      r.status = SDX_LS_INVALID;
      return;
    }
    long long cv = 0, lv = 0;
    const int rc = parse_dec(P, fC.s, fC.e, &cv), rl = parse_dec(P, fL.s, fL.e, &lv);
    if (rc == 2 || rl == 2) {  // int(C) / int(L) raise inside demodulate_mc -> caught, nothing decoded
      r.status = SDX_LS_RAISES;
      return;
    }
    if (rc != 1 || rl != 1) {  // outside the int32 contract (long frames: the general MC kernel)
      r.status = SDX_LS_UNSUPPORTED;
      return;
    }
    out.clock_dev[i] = (int32_t)cv;
    out.mcbitnum_dev[i] = (int32_t)lv;
    out.mcflags_dev[i] = 0;  // msg_data.get("M", "MC") is never "Mc" (mc.py:60); no version
  } else {
    // ---- _parse_to_dict (mu.py:82-94, ms.py:65-78): last value wins, first position counts.
    // P-keys "P<d>" (one digit) go to the lane's LDS table; any longer P-key ("P05", "P10")
    // switches to the general (nested-scan) form below.
    int pos = 0, s, e;
    uint32_t seen = 0;
    uint64_t order = 0;
    int nord = 0;
    bool slow = P.n > 0xFFFF;
    while (next_part(P, pos, s, e)) {
      int eq = -1;
      for (int k = s; k < e; ++k)
        if (P.p[k] == '=') {
          eq = k;
          break;
        }
      const int ke = eq >= 0 ? eq : e;
      const Field f{eq >= 0 ? eq + 1 : e, e};
      if (keq(P, s, ke, "D")) fD = f;
      else if (keq(P, s, ke, "CP")) fCP = f;
      else if (keq(P, s, ke, "SP")) fSP = f;
      else if (keq(P, s, ke, "R")) fR = f;
      else if (keq(P, s, ke, "F")) fF = f;
      else if (P.p[s] == 'P' && ke - s >= 2 && all_digits(P, s + 1, ke)) {
        if (ke - s == 2 && !slow) {
          const int d = P.p[s + 1] - '0';
          if (!((seen >> d) & 1)) {
            seen |= 1u << d;
            order |= (uint64_t)d << (4 * nord);
            ++nord;
          }
          pvt[64 * d] = (uint32_t)f.s | ((uint32_t)f.e << 16);
        } else {
          slow = true;
        }
      }
    }
    if (fD.s < 0) {  // "D" not in msg_data
      r.status = SDX_LS_NODATA;
      return;
    }
    // message_synced.py:21-47 string gates (packing.PulsePacker.add); patterns are converted only
    // where the reference converts them (MS past the gates, MU with non-empty data)
    bool ms_ok = r.kind == SDX_LINE_MS && all_digits(P, fD.s, fD.e) && fCP.s >= 0 && all_digits(P, fCP.s, fCP.e) &&
                 fSP.s >= 0 && all_digits(P, fSP.s, fSP.e) && (fR.s < 0 || all_digits(P, fR.s, fR.e));
    const bool want_pat = r.kind == SDX_LINE_MS ? ms_ok : fD.e > fD.s;
    // _patterns (message_unsynced.py:28-35): id = str(int(k[1:])), value = float(v), ValueError
    // skipped; slot = first successful assignment of the id, value = the last one
    int nslot = 0;
    uint64_t sidp = 0;  // slot z -> id in nibble z
    double* pval = out.pat_val_dev + 10 * (int64_t)i;
    uint8_t* pid = out.pat_id_dev + 10 * (int64_t)i;
    auto assign = [&](int id, double v) {
      int z = 0;
      while (z < nslot && (int)((sidp >> (4 * z)) & 15) != id) ++z;
      if (z == nslot) {
        sidp |= (uint64_t)id << (4 * z);
        pid[z] = (uint8_t)('0' + id);
        ++nslot;
      }
      pval[z] = v;
    };
    if (want_pat && !slow) {
      for (int q = 0; q < nord; ++q) {
        const int d = (int)((order >> (4 * q)) & 15);
        const uint32_t w = pvt[64 * d];
        double v;
        const int rv = parse_pyfloat(P, (int)(w & 0xFFFF), (int)(w >> 16), &v);
        if (rv == 0) continue;  // float() raises ValueError -> skipped
        if (rv == 2) {          // a float outside the exact subset: not modelled
          r.status = SDX_LS_UNSUPPORTED;
          return;
        }
        assign(d, v);
      }
    } else if (want_pat) {
      pos = 0;
      while (next_part(P, pos, s, e)) {
        int eq = -1;
        for (int k = s; k < e; ++k)
          if (P.p[k] == '=') {
            eq = k;
            break;
          }
        const int ke = eq >= 0 ? eq : e;
        if (!(P.p[s] == 'P' && ke - s >= 2 && all_digits(P, s + 1, ke))) continue;
        bool dup = false;  // msg_data holds each key string once, at its first position
        int p2 = 0, s2, e2;
        while (!dup && next_part(P, p2, s2, e2) && s2 < s) {
          int k2 = s2;
          while (k2 < e2 && P.p[k2] != '=') ++k2;
          dup = same_key(P, s, ke, s2, k2);
        }
        if (dup) continue;
        int vs = eq >= 0 ? eq + 1 : e, ve = e;  // ... with the value of its last occurrence
        int p3 = pos, s3, e3;
        while (next_part(P, p3, s3, e3)) {
          int k3 = s3;
          while (k3 < e3 && P.p[k3] != '=') ++k3;
          if (same_key(P, s, ke, s3, k3)) {
            vs = k3 < e3 ? k3 + 1 : e3;
            ve = e3;
          }
        }
        long long idv = 0;
        for (int k = s + 1; k < ke; ++k)
          if (idv < 1000) idv = 10 * idv + (P.p[k] - '0');
        double v;
        const int rv = parse_pyfloat(P, vs, ve, &v);
        if (rv == 0) continue;
        if (rv == 2) {  // a float outside the exact subset
          r.status = SDX_LS_UNSUPPORTED;
          return;
        }
        if (idv >= 10) {  // a multi-character pattern id: the general path (sdx_lines_general)
          gen = true;
          continue;
        }
        assign((int)idv, v);
      }
    }
    if (fD.e - fD.s > SDX_LONG_MAX) gen = true;  // longer than the long variant takes: general path
    out.npat_dev[i] = (uint8_t)nslot;
    if (r.kind == SDX_LINE_MS) {
      int8_t slotv = -1;
      if (ms_ok) {  // str(int(CP)) in the pattern ids, else no demodulation
        long long cp = 0;
        for (int k = fCP.s; k < fCP.e; ++k)
          if (cp < 1000) cp = 10 * cp + (P.p[k] - '0');
        for (int z = 0; z < nslot; ++z)
          if (cp < 10 && (int)((sidp >> (4 * z)) & 15) == cp) slotv = (int8_t)z;
        ms_ok = slotv >= 0;
      }
      out.cp_slot_dev[i] = slotv;
      out.ms_ok_dev[i] = ms_ok ? 1 : 0;
    }
  }
  if ((fR.s >= 0 && fR.e - fR.s > 15) || (fF.s >= 0 && fF.e - fF.s > 15)) {  // meta_dev holds 15 bytes
    r.status = SDX_LS_UNSUPPORTED;
    return;
  }
  r.dS = fD.s;
  r.dE = fD.e;
  r.status = gen ? SDX_LS_GENERAL : SDX_LS_OK;
}

// 16 bytes of meta_dev: value characters, length at byte 15 (255 = absent); the value (<= 15
// bytes) is read as aligned 8-byte words and funnel-shifted
LD uint4 meta16(const Str& P, Field f) {
  if (f.s < 0) return make_uint4(0, 0, 0, 255u << 24);
  const int n = f.e - f.s;
  const uint8_t* q = P.p + f.s;
  const int al = (int)((uintptr_t)q & 7);
  const uint64_t* w = reinterpret_cast<const uint64_t*>(q - al);
  const uint64_t w0 = w[0], w1 = n + al > 8 ? w[1] : 0, w2 = n + al > 16 ? w[2] : 0;
  uint64_t lo = al ? (w0 >> (8 * al)) | (w1 << (64 - 8 * al)) : w0;
  uint64_t hi = al ? (w1 >> (8 * al)) | (w2 << (64 - 8 * al)) : w1;
  if (n < 8) {
    lo &= n ? (~0ull >> (64 - 8 * n)) : 0ull;
    hi = 0;
  } else {
    hi &= n > 8 ? (~0ull >> (64 - 8 * (n - 8))) : 0ull;
  }
  hi = (hi & 0x00FFFFFFFFFFFFFFull) | ((uint64_t)n << 56);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

LD void finish_fields(const Str& P, const LineRes& r, const sdx_lines_out& out, int i) {
  uint4* m = reinterpret_cast<uint4*>(out.meta_dev + 32 * (int64_t)i);
  m[0] = meta16(P, r.fR);
  m[1] = meta16(P, r.fF);
  out.dlen_dev[i] = r.dE - r.dS;
}

constexpr uint8_t ST_RARE = 0xFF;  // internal: compressed, but not recognisably at its first byte

// 6 waves/SIMD: the kernel needs 81 VGPRs unconstrained (5 waves); at 80 it fits 6 with no scratch
__global__ __launch_bounds__(PT) __attribute__((amdgpu_waves_per_eu(6))) void k_parse_lines(sdx_lines in,
                                                                                           sdx_lines_out out) {
  __shared__ uint32_t pv[PT / 64][10 * 64];  // parse_payload's P-key table, per lane
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * PT + threadIdx.x;
  const bool valid = i < in.n;
  uint32_t* pvt = pv[threadIdx.x >> 6] + lane;
  int64_t cp_src = 0, cp_dst = 0;  // uncompressed OK lines: the D characters, copied by the wave
  int cp_len = 0;
#ifdef SDX_LPROF  // k_parse_lines phases: g_lprof slots 10-15 (per wave: max over its lanes)
  unsigned long long lpl[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long* lp = lpl - 10;
#endif
  LP_T(tk0);
#ifndef SDX_NO_LPREFETCH
  {  // The wave's 64 lines are contiguous in bytes_dev: read them once with coalesced 16-byte loads,
     // all in flight together, so that the lane-private byte loads below (strip, header, the fast
     // path's word scans) hit the caches instead of each lane starting its own chain of cold misses
     // (the strip + header checks were 76 % of a wave's cycles, tools/prof_lines.py).  The blocks are
     // 16-byte aligned in the ADDRESS space (whatever the alignment of bytes_dev), so a block holding
     // a byte of the batch lies in that byte's page.
    const int w0i = blockIdx.x * PT + (threadIdx.x & ~63);
    if (w0i < in.n) {
      const int w1i = w0i + 64 < in.n ? w0i + 64 : in.n;
      const uintptr_t a0 = reinterpret_cast<uintptr_t>(in.bytes_dev + in.offsets_dev[w0i]) & ~(uintptr_t)15;
      const uintptr_t a1 = reinterpret_cast<uintptr_t>(in.bytes_dev + in.offsets_dev[w1i]);
      const uint4* base = reinterpret_cast<const uint4*>(a0);
      const int nq = (int)((a1 - a0 + 15) >> 4);
      uint32_t acc = 0;
      for (int q0 = 0; q0 < nq; q0 += 64 * 8) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int q = q0 + u * 64 + lane;
          v[u] = q < nq ? base[q] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].w;
      }
      asm volatile("" ::"v"(acc));  // keeps the loads
    }
  }
#endif
  if (valid) {
    LP_T(tl0);
    const int64_t lo = in.offsets_dev[i], hi = in.offsets_dev[i + 1];
    const uint8_t* L = in.bytes_dev + lo;
    const int len = (int)(hi - lo);
    LineRes r;
    int64_t doff = 3 * lo;
    int plen = -1;
    int a = 0, b = len;  // str.strip() (transport.py:123)
    while (a < b && py_space(L[a])) ++a;
    while (b > a && py_space(L[b - 1])) --b;
    // attempt 0: the fast path on the raw payload (its success implies the framing: every payload
    // byte was checked to be ASCII and not a newline); attempt 1: extract_payload's checks, the
    // decompression, and the general parser
    const bool hdr = b - a >= 6 && L[a] == 0x02 && L[b - 1] == 0x03 && L[a + 1] == 'M' && L[a + 3] == ';' &&
                     L[b - 2] == ';';
    Str P{L + a + 1, b - a - 2};
    const uint8_t t1 = hdr ? up(L[a + 2]) : 0;
    // A payload whose first byte after the header has the high bit set is (the firmware's) Mred=1
    // form: it is left to k_parse_comp (extract_payload's checks, decompression into the slot, the
    // parser), which runs the compressed lines of a batch on full waves.  Other lines reach
    // extract_payload's checks only when the fast path declines (its success implies them: every
    // payload byte was checked to be ASCII and not a newline); one that turns out to be compressed
    // after all goes to k_parse_comp as well.
    const bool likely = hdr && (t1 == 'S' || t1 == 'U' || t1 == 'O' || t1 == 'N') && (L[a + 4] & 0x80);
    const bool comp = false;  // compressed lines are finished by k_parse_comp
    bool decided = !hdr;
    if (likely) {  // Mred=1 form: decompressed and parsed by k_parse_comp with all lanes busy
      r.status = ST_RARE;
      decided = true;
    }
    LP_ADD(10, tl0);
    if (!decided) {
      const uint8_t ty = P.n > 1 ? P.p[1] : 0;
      LP_T(tl1);
      const bool fastok = (ty == 'U' || ty == 'S' || ty == 'C') && fast_payload(P.p, P.n, r, out, i);
      LP_ADD(11, tl1);
      if (!fastok) {
        LP_T(tl2);
        bool c2 = false;
        if (!likely && !frame_check(L, a, b, c2)) {
          r.status = SDX_LS_NOFRAME;
        } else if (c2) {
          r.status = ST_RARE;
        } else {
          parse_payload(P, r, out, i, pvt);
        }
        LP_ADD(12, tl2);
      }
    }
    LP_T(tl3);
    if (r.status == SDX_LS_OK || r.status == SDX_LS_GENERAL) {
      finish_fields(P, r, out, i);
      if (comp) {
        doff = 3 * lo + r.dS;
      } else {
        doff = (3 * lo + 3) & ~3ll;  // word-aligned, inside the slot region (D < line length)
        cp_src = (P.p + r.dS) - in.bytes_dev;
        cp_dst = doff;
        cp_len = r.dE - r.dS;
      }
    }
    LP_ADD(13, tl3);
    out.doff_dev[i] = doff;
    out.plen_dev[i] = plen;
    out.kind_dev[i] = r.kind;
    out.status_dev[i] = r.status;
  }
  LP_T(tl4);
  // the D characters of the wave's uncompressed OK lines, one line at a time: 4 bytes per lane
  // (aligned source words realigned with v_alignbyte), 256 bytes per store instruction
  // Four lines per round: their first 64 words' loads are issued together, then stored (one memory
  // latency per four lines instead of one per line); longer values continue word-strided.
  uint64_t cm = __ballot(cp_len > 0);
  while (cm) {
    constexpr int CB = 4;
    const uint32_t* sw[CB];
    uint32_t* dw[CB];
    int sh[CB], nw[CB];
#pragma unroll
    for (int k = 0; k < CB; ++k) {
      nw[k] = 0;
      sh[k] = 0;
      sw[k] = nullptr;
      dw[k] = nullptr;
      if (cm) {  // wave-uniform
        const int j = __builtin_ctzll(cm);
        cm &= cm - 1;
        const int64_t src = shfl64(cp_src, j);
        sh[k] = (int)(((uintptr_t)in.bytes_dev + src) & 3);
        sw[k] = reinterpret_cast<const uint32_t*>(in.bytes_dev + src - sh[k]);
        dw[k] = reinterpret_cast<uint32_t*>(out.slot_dev + shfl64(cp_dst, j));
        nw[k] = (__shfl(cp_len, j) + 3) >> 2;
      }
    }
    uint32_t lo[CB], hi[CB];
#pragma unroll
    for (int k = 0; k < CB; ++k) {
      lo[k] = hi[k] = 0;
      if (lane < nw[k]) {
        lo[k] = sw[k][lane];
        hi[k] = sw[k][lane + 1];
      }
    }
#pragma unroll
    for (int k = 0; k < CB; ++k) {
      if (lane < nw[k]) dw[k][lane] = __builtin_amdgcn_alignbyte(hi[k], lo[k], sh[k]);
      for (int q = lane + 64; q < nw[k]; q += 64) dw[k][q] = __builtin_amdgcn_alignbyte(sw[k][q + 1], sw[k][q], sh[k]);
    }
  }
  LP_ADD(14, tl4);
  LP_ADD(15, tk0);
#ifdef SDX_LPROF
  for (int k = 0; k < 6; ++k) {
    unsigned long long v = lpl[k];
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long w = __shfl_xor(v, o);
      v = w > v ? w : v;
    }
    if (lane == 0) atomicAdd(&g_lprof[10 + k], v);
  }
#endif
}

// decompress_payload's output goes to the slot (RawFrame.line) and, without the characters of
// the data value, to a lane-private LDS "skeleton": the parse runs on the skeleton, so the payload
// is never read back from the slot.  The data value is all digits (dec_data emits nothing else);
// the skeleton keeps min(n, 2) of them -- every decision fast_payload takes on the value
// (n >= 2 for MU, n >= 1 for MS, digits only) is the same on both -- and its length travels
// beside.  Anything else (a second data part, a skeleton past its buffer, data longer than
// SDX_LONG_MAX, a payload the fast path declines) is parsed from the slot as before.
constexpr int SKEL = 136;  // skeleton bytes per lane (8 * 17: lanes spread over the LDS banks)
#ifdef SDX_NO_SKEL
constexpr bool kSkel = false;  // A/B: parse from the slot
#else
constexpr bool kSkel = true;
#endif
struct SkelWriter {
  Writer8 g;    // the slot
  LdsWriter k;  // the skeleton
  bool in_d = false;
  int nd = 0, dlen = 0;  // data parts, characters of the data value
  int n = 0;
  bool ovf = false;
  // scans read up to 7 bytes past the skeleton's end (the aligned word holding its last byte)
  LD SkelWriter(uint8_t* slot, int cap, uint8_t* skel) : g(slot, cap), k(skel, SKEL - 8) {}
  LD void put(uint8_t c) {
    g.put(c);
    if (!in_d || dlen < 2) k.put(c);
    dlen += in_d ? 1 : 0;
    n = g.n;
    ovf = g.ovf;
  }
  LD void put_uint(uint32_t v) {
    char t[10];
    int q = 0;
    do {
      t[q++] = (char)('0' + v % 10);
      v /= 10;
    } while (v);
    while (q) put((uint8_t)t[--q]);
  }
  LD void put8(uint64_t x) {
    if (!in_d || dlen < 2) {  // the skeleton takes (some of) these
      for (int t = 0; t < 8; ++t) put((uint8_t)(x >> (8 * t)));
      return;
    }
    g.put8(x);
    dlen += 8;
    n = g.n;
    ovf = g.ovf;
  }
  LD void mark_d(bool on) {
    in_d = on;
    if (on) {
      ++nd;
      dlen = 0;
    }
  }
  LD void finish() { g.finish(); }
};

// one compressed line (ST_RARE): extract_payload's checks, decompress_payload into the line's slot
// (and the skeleton), then the fast path on the skeleton, or on the slot with the general parser
// behind it
LD void parse_compressed(const sdx_lines& in, const sdx_lines_out& out, int i, uint32_t* pvt, uint8_t* skel LP_ARG) {
  LP_T(t0);
  const int64_t lo = in.offsets_dev[i];
  const int len = (int)(in.offsets_dev[i + 1] - lo);
  const uint8_t* L = in.bytes_dev + lo;
  int a = 0, b = len;
  while (a < b && py_space(L[a])) ++a;
  while (b > a && py_space(L[b - 1])) --b;
  LineRes r;
  int plen = -1;
  int64_t doff = 3 * lo;
  bool comp = false;
  const bool framed = frame_check(L, a, b, comp);
  LP_ADD(1, t0);
  if (!framed) {
    r.status = SDX_LS_NOFRAME;
  } else {  // comp holds: the first payload byte, or another one, has the high bit set
    LP_T(t1);
    SkelWriter w(out.slot_dev + 3 * lo, 3 * len, skel);
    const bool dec = decompress(Str{L + a + 1, b - a - 2}, w);
    LP_ADD(2, t1);
    if (!(dec && !w.g.ovf)) {
      r.status = SDX_LS_UNSUPPORTED;
    } else {
      plen = w.g.n;
      const Str P{out.slot_dev + 3 * lo, w.g.n};
      const Str K{skel, w.k.n};
      const uint8_t ty = K.n > 1 ? K.p[1] : 0;
      LP_T(t2);
      bool fast = false;
      if (kSkel && !w.k.ovf && w.nd == 1 && w.dlen <= SDX_LONG_MAX && (ty == 'U' || ty == 'S') && fast_payload(K.p, K.n, r, out, i)) {
        fast = true;
        r.dE = r.dS + w.dlen;  // the data value's real extent (its position is the skeleton's)
        finish_fields(K, r, out, i);
        doff = 3 * lo + r.dS;
      }
      LP_ADD(3, t2);
      if (!fast) {
        LP_T(t3);
        r = LineRes{};
        const uint8_t tp = P.n > 1 ? P.p[1] : 0;
        if (!((tp == 'U' || tp == 'S' || tp == 'C') && fast_payload(P.p, P.n, r, out, i))) parse_payload(P, r, out, i, pvt);
        if (r.status == SDX_LS_OK || r.status == SDX_LS_GENERAL) {
          finish_fields(P, r, out, i);
          doff = 3 * lo + r.dS;
        }
        LP_ADD(4, t3);
#ifdef SDX_LPROF
        lp[8] += 1;
#endif
      }
    }
  }
  LP_T(t5);
  out.doff_dev[i] = doff;
  out.plen_dev[i] = plen;
  out.kind_dev[i] = r.kind;
  out.status_dev[i] = r.status;
  LP_ADD(6, t5);
#ifdef SDX_LPROF
  lp[9] += 1;
#endif
}

// the lines k_parse_lines left to it (ST_RARE): each wave scans `chunk` lines (a multiple of 64),
// queues the compressed ones in LDS and parses them 64 at a time (lane = line), so the
// decompression work of the ~20 % compressed lines of a mixed stream runs on full waves.  A wave's
// time is about one line's serial decompress + parse, so the host sizes `chunk` for the grid to fit
// the GPU's resident waves in one round (comp_chunk below).  Measured alternative: staging the raw
// lines and the decompressed payloads in 38 KB of LDS per wave (1 wave/SIMD) ran 1.74 vs 1.13 ms
// for the parse (profiles/r03/lines_comp_ab.log): the per-lane work is issue-bound, and needs
// the 4 waves/SIMD this layout keeps.
constexpr int COMP_CHUNK = 192;         // lower bound of the chunk (~40 compressed at the bench mix)
constexpr int COMP_WAVES_PER_CU = 16;   // 4 waves/SIMD (VGPRs; LDS 36.8 KB per 4-wave block)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_parse_comp(sdx_lines in, sdx_lines_out out, int chunk) {
  __shared__ int q[4][128];
  __shared__ uint64_t sk[4][64][SKEL / 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* skel = reinterpret_cast<uint8_t*>(sk[wave][lane]);
  // parse_payload's P-key table (10 x 64 words per wave) aliases the wave's skeletons: it is used
  // only after every lane of the wave has left its skeleton (parse_compressed's second block)
  static_assert(10 * 64 * 4 <= 64 * SKEL, "the P-key table fits the wave's skeletons");
  uint32_t* pvt = reinterpret_cast<uint32_t*>(sk[wave]) + lane;
#ifdef SDX_LPROF
  unsigned long long lp[16] = {};
  const unsigned long long tk0 = __builtin_amdgcn_s_memtime();
#endif
  const int64_t base = ((int64_t)blockIdx.x * 4 + wave) * chunk;
  int qn = 0;
  for (int c = 0; c < chunk; c += 64) {
    const int64_t i = base + c + lane;
    const bool rare = i < in.n && out.status_dev[i] == ST_RARE;
    const uint64_t m = __ballot(rare);
    if (rare) q[wave][qn + __popcll(m & ((1ull << lane) - 1))] = (int)i;
    qn += __popcll(m);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (qn >= 64) {
      const int li = q[wave][lane];
      const int rest = lane < qn - 64 ? q[wave][64 + lane] : 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane < qn - 64) q[wave][lane] = rest;
      qn -= 64;
      parse_compressed(in, out, li, pvt, skel LP_PASS);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (lane < qn) parse_compressed(in, out, q[wave][lane], pvt, skel LP_PASS);
#ifdef SDX_LPROF
  lp[0] = __builtin_amdgcn_s_memtime() - tk0;  // the wave's whole time
#pragma unroll
  for (int k = 0; k < 16; ++k) {  // phases: max over lanes (the wave runs while any lane does); counts: sum
    unsigned long long v = lp[k];
    for (int o = 32; o; o >>= 1) {
      const unsigned long long y = (unsigned long long)__shfl_xor((long long)v, o);
      v = k >= 8 ? v + y : (y > v ? y : v);
    }
    if (lane == 0) atomicAdd(&g_lprof[k], v);
  }
#endif
}

// lines per k_parse_comp wave: at least COMP_CHUNK, and enough that the grid's waves fit the
// device's resident waves in one round
int comp_chunk(int n) {
  int dev = 0, cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cu <= 0)
    cu = 256;
  const int64_t waves = (int64_t)cu * COMP_WAVES_PER_CU;
  int64_t c = ((int64_t)n + waves - 1) / waves;
  c = (c + 63) / 64 * 64;
  return (int)(c < COMP_CHUNK ? COMP_CHUNK : c);
}

// ---- selection lists (sdx_select_lines): class of a parsed line, -1 = not demodulated
LD int sel_class(const sdx_lines_out& o, int i) {
  if (o.status_dev[i] != SDX_LS_OK) return -1;
  const uint8_t k = o.kind_dev[i];
  const int32_t n = o.dlen_dev[i];
  if (k == SDX_LINE_MU) return n <= SDX_SHORT_MAX ? SDX_SEL_MU_SHORT : SDX_SEL_MU_LONG;
  if (k == SDX_LINE_MS) {
    if (!o.ms_ok_dev[i]) return -1;
    return n <= SDX_SHORT_MAX ? SDX_SEL_MS_SHORT : SDX_SEL_MS_LONG;
  }
  if (k == SDX_LINE_MC) return n <= SDX_MC_SHORT_HEX ? SDX_SEL_MC : SDX_SEL_MC_LONG;
  if (k == SDX_LINE_MN) return SDX_SEL_MN;
  return -1;
}

constexpr int SEL_THREADS = 256;
static_assert(SDX_SEL_CHUNK % SEL_THREADS == 0, "chunk = whole rounds of the workgroup");

// per-chunk class counts -> scratch[chunk * 8 + class]
__global__ __launch_bounds__(SEL_THREADS) void k_sel_count(sdx_lines_out o, int n, int32_t* scratch) {
  __shared__ int32_t c[SDX_SEL_NCLASS];
  if (threadIdx.x < SDX_SEL_NCLASS) c[threadIdx.x] = 0;
  __syncthreads();
  int mine[SDX_SEL_NCLASS] = {};
  const int base = blockIdx.x * SDX_SEL_CHUNK;
  for (int r = 0; r < SDX_SEL_CHUNK; r += SEL_THREADS) {
    const int i = base + r + threadIdx.x;
    const int k = i < n ? sel_class(o, i) : -1;
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q) mine[q] += k == q;
  }
#pragma unroll
  for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
    int v = mine[q];
    for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&c[q], v);
  }
  __syncthreads();
  if (threadIdx.x < 8) scratch[blockIdx.x * 8 + threadIdx.x] = threadIdx.x < SDX_SEL_NCLASS ? c[threadIdx.x] : 0;
}

// ordered write: chunk b's entries of class k go to start_k + (class-k lines of chunks < b) + rank in chunk
__global__ __launch_bounds__(SEL_THREADS) void k_sel_write(sdx_lines_out o, int n, int nchunk,
                                                           const int32_t* scratch, int32_t* sel, int32_t* counts) {
  __shared__ int32_t tot[SDX_SEL_NCLASS], pre[SDX_SEL_NCLASS], wcnt[SEL_THREADS / 64][SDX_SEL_NCLASS];
  if (threadIdx.x < SDX_SEL_NCLASS) tot[threadIdx.x] = pre[threadIdx.x] = 0;
  __syncthreads();
  {
    int t[SDX_SEL_NCLASS] = {}, p[SDX_SEL_NCLASS] = {};
    for (int b = threadIdx.x; b < nchunk; b += SEL_THREADS)
#pragma unroll
      for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
        const int v = scratch[b * 8 + q];
        t[q] += v;
        if (b < (int)blockIdx.x) p[q] += v;
      }
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
      int a = t[q], c = p[q];
      for (int d = 32; d; d >>= 1) {
        a += __shfl_xor(a, d);
        c += __shfl_xor(c, d);
      }
      if ((threadIdx.x & 63) == 0) {
        if (a) atomicAdd(&tot[q], a);
        if (c) atomicAdd(&pre[q], c);
      }
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < 8) counts[threadIdx.x] = threadIdx.x < SDX_SEL_NCLASS ? tot[threadIdx.x] : 0;
  int cur[SDX_SEL_NCLASS];  // next free position of each class for this chunk (uniform)
  {
    int st = 0;
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
      cur[q] = st + pre[q];
      st += tot[q];
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int base = blockIdx.x * SDX_SEL_CHUNK;
  for (int r = 0; r < SDX_SEL_CHUNK; r += SEL_THREADS) {
    const int i = base + r + threadIdx.x;
    const int k = i < n ? sel_class(o, i) : -1;
    uint64_t m[SDX_SEL_NCLASS];
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
      m[q] = __ballot(k == q);
      if (lane == 0) wcnt[wave][q] = __popcll(m[q]);
    }
    __syncthreads();
    if (k >= 0) {
      int pos = 0;
#pragma unroll
      for (int q = 0; q < SDX_SEL_NCLASS; ++q)
        if (q == k) {
          pos = cur[q] + __popcll(m[q] & lt);
          for (int w = 0; w < wave; ++w) pos += wcnt[w][q];
        }
      sel[pos] = i;
    }
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q)
      for (int w = 0; w < SEL_THREADS / 64; ++w) cur[q] += wcnt[w][q];
    __syncthreads();
  }
}

// ---- sdx_lines_general: the general-path batch of the SDX_LS_GENERAL lines (lane = line) --------
// _parse_to_dict (mu.py:82-94, ms.py:65-78: first position, last value) and _patterns
// (message_unsynced.py:28-35: id = str(int(key[1:])), float(value), ValueError skipped) with ids as
// strings, the MS string gates and str(int(CP)) (message_synced.py:21-57).
constexpr int GEN_P = SDX_GEN_MAXPAT, GEN_ID = SDX_GEN_IDSTR;

// the key's digits with leading zeros removed (str(int(digits)) for ASCII digits); false if > 15
LD bool id_string(const Str& P, int s, int e, uint8_t* dst) {
  while (s < e - 1 && P.p[s] == '0') ++s;
  if (e - s > GEN_ID - 1) return false;
  dst[0] = (uint8_t)(e - s);
  for (int k = s; k < e; ++k) dst[1 + k - s] = P.p[k];
  return true;
}

__global__ __launch_bounds__(64) void k_lines_general(sdx_lines in, sdx_lines_out out, const int32_t* sel, int n_sel,
                                                      sdx_lines_general_out g) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= n_sel) return;
  const int i = sel[j];
  const int64_t lo = in.offsets_dev[i];
  const int len = (int)(in.offsets_dev[i + 1] - lo);
  Str P;
  if (out.plen_dev[i] >= 0) {  // decompressed into the slot
    P = Str{out.slot_dev + 3 * lo, out.plen_dev[i]};
  } else {  // the stripped line between STX and ETX (frame_check passed in sdx_parse_lines)
    const uint8_t* L = in.bytes_dev + lo;
    int a = 0, b = len;
    while (a < b && py_space(L[a])) ++a;
    while (b > a && py_space(L[b - 1])) --b;
    P = Str{L + a + 1, b - a - 2};
  }
  g.offsets_dev[j] = out.doff_dev[i];
  g.len_dev[j] = out.dlen_dev[i];
  uint8_t* ids = g.pat_ids_dev + (int64_t)j * GEN_P * GEN_ID;
  double* vals = g.pat_val_dev + (int64_t)j * GEN_P;
  Field fD{-1, -1}, fCP{-1, -1}, fSP{-1, -1}, fR{-1, -1};
  int pos = 0, s, e;
  while (next_part(P, pos, s, e)) {
    int k = s;
    while (k < e && P.p[k] != '=') ++k;
    const Field f{k < e ? k + 1 : e, e};
    if (keq(P, s, k, "D")) fD = f;
    else if (keq(P, s, k, "CP")) fCP = f;
    else if (keq(P, s, k, "SP")) fSP = f;
    else if (keq(P, s, k, "R")) fR = f;
  }
  const bool ms = out.kind_dev[i] == SDX_LINE_MS;
  bool ms_ok = ms && fD.s >= 0 && all_digits(P, fD.s, fD.e) && fCP.s >= 0 && all_digits(P, fCP.s, fCP.e) &&
               fSP.s >= 0 && all_digits(P, fSP.s, fSP.e) && (fR.s < 0 || all_digits(P, fR.s, fR.e));
  const bool want = ms ? ms_ok : (fD.s >= 0 && fD.e > fD.s);
  int np = 0;
  bool bad = false;
  pos = 0;
  while (want && !bad && next_part(P, pos, s, e)) {
    int ke = s;
    while (ke < e && P.p[ke] != '=') ++ke;
    if (!(P.p[s] == 'P' && ke - s >= 2 && all_digits(P, s + 1, ke))) continue;
    bool dup = false;  // msg_data holds each key string once, at its first position ...
    int p2 = 0, s2, e2;
    while (!dup && next_part(P, p2, s2, e2) && s2 < s) {
      int k2 = s2;
      while (k2 < e2 && P.p[k2] != '=') ++k2;
      dup = same_key(P, s, ke, s2, k2);
    }
    if (dup) continue;
    int vs = ke < e ? ke + 1 : e, ve = e;  // ... with the value of its last occurrence
    int p3 = pos, s3, e3;
    while (next_part(P, p3, s3, e3)) {
      int k3 = s3;
      while (k3 < e3 && P.p[k3] != '=') ++k3;
      if (same_key(P, s, ke, s3, k3)) {
        vs = k3 < e3 ? k3 + 1 : e3;
        ve = e3;
      }
    }
    double v;
    const int rv = parse_pyfloat(P, vs, ve, &v);
    if (rv == 0) continue;  // float() raises ValueError: key skipped
    uint8_t id[GEN_ID];
    if (rv == 2 || !id_string(P, s + 1, ke, id)) {
      bad = true;
      break;
    }
    int z = 0;  // pats[id] = value: first assignment fixes the slot, the last one the value
    for (; z < np; ++z) {
      bool same = ids[z * GEN_ID] == id[0];
      for (int q = 1; same && q <= id[0]; ++q) same = ids[z * GEN_ID + q] == id[q];
      if (same) break;
    }
    if (z == np) {
      if (np == GEN_P) {
        bad = true;
        break;
      }
      for (int q = 0; q <= id[0]; ++q) ids[z * GEN_ID + q] = id[q];
      ++np;
    }
    vals[z] = v;
  }
  int8_t cp = -1;
  if (!bad && ms && ms_ok) {  // str(int(CP)) in the pattern ids
    uint8_t id[GEN_ID];
    if (id_string(P, fCP.s, fCP.e, id)) {
      for (int z = 0; z < np && cp < 0; ++z) {
        bool same = ids[z * GEN_ID] == id[0];
        for (int q = 1; same && q <= id[0]; ++q) same = ids[z * GEN_ID + q] == id[q];
        if (same) cp = (int8_t)z;
      }
    }
    ms_ok = cp >= 0;
  }
  if (bad) {
    out.status_dev[i] = SDX_LS_UNSUPPORTED;
    np = 0;
    ms_ok = false;
  }
  g.npat_dev[j] = (uint8_t)np;
  g.cp_slot_dev[j] = cp;
  g.ms_ok_dev[j] = ms_ok ? 1 : 0;
}

}  // namespace sdxl

extern "C" int sdx_select_lines(const sdx_lines_out* out, int32_t n, int32_t* sel_dev, int32_t* counts_dev,
                                int32_t* scratch_dev, void* hip_stream) {
  if (!out || n < 0 || !counts_dev) return sdx::set_error(SDX_EINVAL, "sdx_select_lines: bad arguments");
  hipStream_t st = (hipStream_t)hip_stream;
  if (n == 0) {
    const hipError_t e = hipMemsetAsync(counts_dev, 0, 8 * sizeof(int32_t), st);
    return e == hipSuccess ? SDX_OK : sdx::set_error(SDX_EHIP, "sdx_select_lines: memset failed");
  }
  if (!sel_dev || !scratch_dev || !out->kind_dev || !out->status_dev || !out->dlen_dev || !out->ms_ok_dev)
    return sdx::set_error(SDX_EINVAL, "sdx_select_lines: null buffer");
  const int nchunk = (n + SDX_SEL_CHUNK - 1) / SDX_SEL_CHUNK;
  hipLaunchKernelGGL(sdxl::k_sel_count, dim3(nchunk), dim3(sdxl::SEL_THREADS), 0, st, *out, n, scratch_dev);
  hipLaunchKernelGGL(sdxl::k_sel_write, dim3(nchunk), dim3(sdxl::SEL_THREADS), 0, st, *out, n, nchunk,
                     (const int32_t*)scratch_dev, sel_dev, counts_dev);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("sdx_select_lines: ") + hipGetErrorString(e));
  return SDX_OK;
}

#ifdef SDX_LPROF
extern "C" int sdx_lprof_read(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(sdxl::g_lprof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(sdxl::g_lprof), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

extern "C" int sdx_parse_lines(const sdx_lines* lines, const sdx_lines_out* out, void* hip_stream) {
  if (!lines || !out || lines->n < 0) return sdx::set_error(SDX_EINVAL, "sdx_parse_lines: bad arguments");
  if (lines->n == 0) return SDX_OK;
  if (!lines->bytes_dev || !lines->offsets_dev || !out->kind_dev || !out->status_dev || !out->slot_dev ||
      !out->doff_dev || !out->dlen_dev || !out->npat_dev || !out->pat_id_dev || !out->pat_val_dev ||
      !out->cp_slot_dev || !out->ms_ok_dev || !out->clock_dev || !out->mcbitnum_dev || !out->mcflags_dev ||
      !out->meta_dev || !out->plen_dev)
    return sdx::set_error(SDX_EINVAL, "sdx_parse_lines: null buffer");
  if (((uintptr_t)out->meta_dev & 15) != 0)
    return sdx::set_error(SDX_EINVAL, "sdx_parse_lines: meta_dev must be 16-byte aligned");
  if (((uintptr_t)lines->bytes_dev & 7) != 0 || ((uintptr_t)out->slot_dev & 7) != 0)
    return sdx::set_error(SDX_EINVAL, "sdx_parse_lines: bytes_dev and slot_dev must be 8-byte aligned");
  const int grid = (lines->n + sdxl::PT - 1) / sdxl::PT;
  hipLaunchKernelGGL(sdxl::k_parse_lines, dim3(grid), dim3(sdxl::PT), 0, (hipStream_t)hip_stream, *lines, *out);
  const int chunk = sdxl::comp_chunk(lines->n);
  hipLaunchKernelGGL(sdxl::k_parse_comp, dim3((int)(((int64_t)lines->n + 4 * chunk - 1) / (4 * chunk))), dim3(256), 0,
                     (hipStream_t)hip_stream, *lines, *out, chunk);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("sdx_parse_lines: ") + hipGetErrorString(e));
  return SDX_OK;
}

extern "C" int sdx_lines_general(const sdx_lines* lines, const sdx_lines_out* out, const int32_t* sel_dev, int32_t n_sel,
                                 const sdx_lines_general_out* gen, void* hip_stream) {
  if (!lines || !out || !gen || n_sel < 0) return sdx::set_error(SDX_EINVAL, "sdx_lines_general: bad arguments");
  if (n_sel == 0) return SDX_OK;
  if (!sel_dev || !gen->offsets_dev || !gen->len_dev || !gen->npat_dev || !gen->pat_ids_dev || !gen->pat_val_dev ||
      !gen->cp_slot_dev || !gen->ms_ok_dev)
    return sdx::set_error(SDX_EINVAL, "sdx_lines_general: null buffer");
  hipLaunchKernelGGL(sdxl::k_lines_general, dim3((n_sel + 63) / 64), dim3(64), 0, (hipStream_t)hip_stream, *lines, *out,
                     sel_dev, n_sel, *gen);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("sdx_lines_general: ") + hipGetErrorString(e));
  return SDX_OK;
}
